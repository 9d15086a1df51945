#!/bin/bash
# Weight-gradient GEMMs on a side stream under a HIGH-priority compute stream (gap filling) vs defaults.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for v in "0 0" "1 1" "1 0" "0 1"; do
    set -- $v
    SFTAMD_WGRAD_STREAM=$1 SFTAMD_COMPUTE_PRIO=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_45_b.log 2>&1 || { tail -30 gpurun_out/r2_45_b.log; exit 1; }
    echo "WGRAD_STREAM=$1 PRIO=$2 $(tail -1 gpurun_out/r2_45_b.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["final_loss"])')"
  done
done
