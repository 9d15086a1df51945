#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad" > gpurun_out/t13w.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t13w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/bw13.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bw13.log; ok $rc
timeout -k 10 300 python -m pytest tests/test_generation_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -k "decode or graph" > gpurun_out/t13g.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t13g.log; ok $rc
