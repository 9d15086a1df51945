#!/bin/bash
# round 6: LoRA step with plain input gradients on the 8-wave ring (default) vs the 4-wave ring (SFTAMD_DGRAD_RING8=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for r in 1 0; do
SFTAMD_DGRAD_RING8=$r timeout -k 10 300 python -u bench.py --freeze-policy lora --steps 20 > gpurun_out/r6_67_l${r}_$i.log 2>&1 || { tail -20 gpurun_out/r6_67_l${r}_$i.log; exit 1; }
echo "lora ring8=$r $i: $(v gpurun_out/r6_67_l${r}_$i.log)"
done
done
