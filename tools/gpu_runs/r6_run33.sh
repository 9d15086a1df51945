#!/bin/bash
# round 6: the headline step with R CUs held on a side stream for 100 ms of every step (RCCL stand-in)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_33.log; : > $out
for r in 0 8 0 8 32; do
  SFTAMD_BENCH_HOG_CUS=$r timeout -k 10 300 python bench.py > gpurun_out/r6_33_b.log 2>&1 || { tail -20 gpurun_out/r6_33_b.log; exit 1; }
  echo "held=$r $(tail -1 gpurun_out/r6_33_b.log | cut -c1-150)" >> $out
done
cat $out
