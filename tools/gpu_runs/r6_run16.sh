#!/bin/bash
# round 6: the 4-wave kernel with an LDS-staged SwiGLU-backward epilogue (dgrad cfg 14 + gu) vs cfg 7: correctness,
# microbench (down + SwiGLU bwd at M = 8192), in-step A/B via SFTAMD_SWIGLU_DGRAD_CFG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py -k "dgrad" > gpurun_out/r6_16_tests.log 2>&1 || { tail -40 gpurun_out/r6_16_tests.log; exit 1; }
tail -2 gpurun_out/r6_16_tests.log
for r in 1 2; do
DGRAD_CFGS=7,14 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r6_16_dgrad$r.log 2>&1 || { tail -30 gpurun_out/r6_16_dgrad$r.log; exit 1; }
grep swiglu gpurun_out/r6_16_dgrad$r.log
done
