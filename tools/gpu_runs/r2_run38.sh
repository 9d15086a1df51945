#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for p in 1 0; do
    SFTAMD_COMPUTE_PRIO=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_38_b$p.log 2>&1 || { tail -30 gpurun_out/r2_38_b$p.log; exit 1; }
    echo "PRIO=$p $(tail -1 gpurun_out/r2_38_b$p.log | cut -c1-140)"
  done
done
