#!/bin/bash
# round 5: end-to-end A/B of the row-contiguous forward GEMM routing (interleaved x2) + step profile of the fused arm
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_02_$n.log 2>&1 || { tail -20 gpurun_out/r5_02_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r5_02_$n.log)"
}
for r in 1 2; do
  run base$r SFTAMD_TN=rope SFTAMD_TN_CFG=11
  run rope61_$r SFTAMD_TN=rope
  run both61_$r SFTAMD_TN=1
  run all61_$r SFTAMD_TN=1 SFTAMD_FWD_HIP_MAXN=4096
done
SFTAMD_TN=1 SFTAMD_FWD_HIP_MAXN=4096 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof02 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r5_02_p.log 2>&1 || { tail -20 gpurun_out/r5_02_p.log; exit 1; }
db=$(ls /tmp/prof02/*/run_results.db /tmp/prof02/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r5_02_step_prof.md > /dev/null
head -30 gpurun_out/r5_02_step_prof.md
