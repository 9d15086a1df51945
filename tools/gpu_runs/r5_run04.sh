#!/bin/bash
# round 5: is the in-step loss of the fused gate_up + SwiGLU kernel an overlap (AdamW) interaction? base vs both61 with
# and without the overlapped update, interleaved x2, then a per-kernel step profile of both61 --no-overlap
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env..., -- bench args
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r5_04_$n.log 2>&1 || { tail -20 gpurun_out/r5_04_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r5_04_$n.log)"
}
for r in 1 2; do
  run base$r SFTAMD_TN=rope SFTAMD_TN_CFG=11 --
  run both61_$r SFTAMD_TN=1 --
  run base_no$r SFTAMD_TN=rope SFTAMD_TN_CFG=11 -- --no-overlap
  run both61_no$r SFTAMD_TN=1 -- --no-overlap
done
for arm in base both; do
  if [ $arm = base ]; then E="SFTAMD_TN=rope SFTAMD_TN_CFG=11"; else E="SFTAMD_TN=1"; fi
  env $E timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof04$arm -o run -- python bench.py --steps 6 --warmup 2 --no-overlap > gpurun_out/r5_04_p$arm.log 2>&1 || { tail -20 gpurun_out/r5_04_p$arm.log; exit 1; }
  db=$(ls /tmp/prof04$arm/*/run_results.db /tmp/prof04$arm/run_results.db 2>/dev/null | head -1)
  python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_04_step_prof_$arm.md > /dev/null
done
head -24 gpurun_out/r5_04_step_prof_both.md
