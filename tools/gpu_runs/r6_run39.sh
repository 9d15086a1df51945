#!/bin/bash
# round 6: the down projection's weight gradient on a side stream, concurrent with the SwiGLU-fused input gradient
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_39.log; : > $out
for v in 1 0 1 0 1 0; do
  SFTAMD_WGRAD_SIDE=$v timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r6_39_b.log 2>&1 || { tail -20 gpurun_out/r6_39_b.log; exit 1; }
  echo "side=$v $(tail -1 gpurun_out/r6_39_b.log | cut -c60-150) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r6_39_b.log)" >> $out
done
cat $out
