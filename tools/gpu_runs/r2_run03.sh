#!/bin/bash
# Round 2: split-K wgrad correctness + microbench for the small-grid weight gradients (o_proj, qkv, down).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/r2_03_tests.log 2>&1 || { tail -40 gpurun_out/r2_03_tests.log; exit 1; }
tail -2 gpurun_out/r2_03_tests.log
timeout -k 10 300 python tools/bench_wgrad.py --only o,qkv,down --cfgs 9,10,209,210,409,410,809 > gpurun_out/r2_03_wgrad.log 2>&1 || { tail -20 gpurun_out/r2_03_wgrad.log; exit 1; }
cat gpurun_out/r2_03_wgrad.log
