#!/bin/bash
# round 6: weight gradients on a side stream, concurrent with the node's input gradient, per site (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_40.log; : > $out
for rep in 1 2; do
for v in 0 down down,gate_up down,o,qkv down,lm_head all; do
  SFTAMD_WGRAD_SIDE=$v timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r6_40_b.log 2>&1 || { tail -20 gpurun_out/r6_40_b.log; exit 1; }
  echo "side=$v $(grep -o '"value": [0-9.]*' gpurun_out/r6_40_b.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r6_40_b.log)" >> $out
done
done
cat $out
