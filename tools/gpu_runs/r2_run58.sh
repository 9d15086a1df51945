#!/bin/bash
# Re-tune of the launch knobs after the round's kernel changes: tile-group width of the TN / NN GEMMs, dgrad tail
# split, fused-Adam grid. Interleaved bench A/B on one box (20 timed steps each).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_58_$tag.log 2>&1 || { tail -30 gpurun_out/r2_58_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r2_58_$tag.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["final_loss"])')"
}
for i in 1 2; do
  run base$i SFTAMD_NOOP=1
  run tn_group4_$i SFTAMD_TN_GROUP=4
  run tn_group16_$i SFTAMD_TN_GROUP=16
  run dgrad_group4_$i SFTAMD_DGRAD_GROUP=4
  run dgrad_group16_$i SFTAMD_DGRAD_GROUP=16
  run dgrad_tail3_$i SFTAMD_DGRAD_TAIL=3
done
