#!/bin/bash
# Round 2: attention forward at 4 waves/SIMD (launch bounds) — tests + microbench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 120 --timeout-method thread > gpurun_out/r2_19_tests.log 2>&1 || { tail -40 gpurun_out/r2_19_tests.log; exit 1; }
tail -1 gpurun_out/r2_19_tests.log
B=16 ATTN_QUICK=1 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/r2_19_attn.log 2>&1 || { tail -20 gpurun_out/r2_19_attn.log; exit 1; }
grep impl gpurun_out/r2_19_attn.log
