#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad or rmsnorm" > gpurun_out/t20.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wgrad.py --cfgs 7,10,9,11 --only qkv,gate_up,down,lm_head > gpurun_out/bw20.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bw20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b20.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b20.log
