#!/bin/bash
# Fused gradient norm (wgrad epilogue partials + leftover chunks): tests, then same-box A/B vs the previous commit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "norm_slots or sumsq_chunks or wgrad_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_28_tests.log 2>&1 || { tail -40 gpurun_out/r2_28_tests.log; exit 1; }
tail -1 gpurun_out/r2_28_tests.log
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -k "fused_grad_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_28_tests2.log 2>&1 || { tail -40 gpurun_out/r2_28_tests2.log; exit 1; }
tail -1 gpurun_out/r2_28_tests2.log
R=3 bash tools/gpu_runs/r2_ab.sh
