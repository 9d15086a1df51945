#!/bin/bash
# BK64 256x128 forward GEMM (3 / 2 LDS stages): numerics, then the microbench against hipBLASLt and the other tiles.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t54.log 2>&1 || { tail -30 gpurun_out/t54.log; exit 1; }
tail -2 gpurun_out/t54.log
timeout -k 10 400 python tools/bench_gemm_tn.py > gpurun_out/g54.log 2>&1 || { tail -20 gpurun_out/g54.log; exit 1; }
grep -v Warning gpurun_out/g54.log
