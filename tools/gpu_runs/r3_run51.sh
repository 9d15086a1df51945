#!/bin/bash
# 4-wave SwiGLU dgrad with the LDS-staged epilogue: tests, dgrad microbench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py -k "4wave or dgrad or wgrad" \
  > gpurun_out/r3_51_test.log 2>&1 || { tail -40 gpurun_out/r3_51_test.log; exit 1; }
tail -1 gpurun_out/r3_51_test.log
DGRAD_CFGS=7,12,13 timeout -k 10 200 python -u tools/bench_dgrad.py > gpurun_out/r3_51_dg.log 2>&1 || { tail -30 gpurun_out/r3_51_dg.log; exit 1; }
grep -v "^\[" gpurun_out/r3_51_dg.log | tail -6
