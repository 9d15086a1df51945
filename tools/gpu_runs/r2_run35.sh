#!/bin/bash
# GQA-grouped dK/dV (bwd_dkdv5_kernel): flash tests, attention microbench, bench.py A/B vs per-head + reduce.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_35_tests.log 2>&1 || { tail -40 gpurun_out/r2_35_tests.log; exit 1; }
tail -1 gpurun_out/r2_35_tests.log
B=16 ATTN_QUICK=1 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/r2_35_attn.log 2>&1 || { tail -30 gpurun_out/r2_35_attn.log; exit 1; }
cat gpurun_out/r2_35_attn.log
for i in 1 2; do
  for g in 1 0; do
    SFTAMD_ATTN_GQA=$g timeout -k 10 300 python bench.py > gpurun_out/r2_35_b$g.log 2>&1 || { tail -30 gpurun_out/r2_35_b$g.log; exit 1; }
    echo "GQA=$g $(tail -1 gpurun_out/r2_35_b$g.log | cut -c1-140)"
  done
done
