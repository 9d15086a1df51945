#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad" > gpurun_out/t18w.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t18w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wgrad.py --cfgs 1,3,4,7,8,9 > gpurun_out/bw18.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bw18.log
