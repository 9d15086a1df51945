#!/bin/bash
# Round 2: hand-written NN dgrad GEMM (+ fused SwiGLU backward): correctness + microbench vs hipBLASLt.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k dgrad --timeout 120 --timeout-method thread > gpurun_out/r2_08_tests.log 2>&1 || { tail -40 gpurun_out/r2_08_tests.log; exit 1; }
tail -1 gpurun_out/r2_08_tests.log
timeout -k 10 300 python tools/bench_dgrad.py > gpurun_out/r2_08_dgrad.log 2>&1 || { tail -20 gpurun_out/r2_08_dgrad.log; exit 1; }
grep shape gpurun_out/r2_08_dgrad.log
