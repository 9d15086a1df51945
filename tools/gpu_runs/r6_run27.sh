#!/bin/bash
# round 6: interleaved same-box A/B of the delta hand-off (SFTAMD_ATTN_DELTA=1 default vs 0 = the delta kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_27_ab.log; : > $out
for i in 1 2 3; do
  for v in 1 0; do
    SFTAMD_ATTN_DELTA=$v timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r6_27_b.log 2>&1 || { tail -20 gpurun_out/r6_27_b.log; exit 1; }
    echo "delta_fused=$v $(tail -1 gpurun_out/r6_27_b.log | cut -c1-160)" >> $out
  done
done
cat $out
