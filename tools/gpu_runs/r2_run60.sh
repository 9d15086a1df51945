#!/bin/bash
# Cross-entropy kernel isolated A/B (1 vs 4 row loads in flight per thread).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for u in 1 4 1 4; do
  SFTAMD_CE_UNROLL=$u timeout -k 10 120 python tools/bench_ce.py > gpurun_out/r2_60_ce$u.log 2>&1 || { tail -20 gpurun_out/r2_60_ce$u.log; exit 1; }
  echo "CE_UNROLL=$u $(tail -1 gpurun_out/r2_60_ce$u.log)"
done
