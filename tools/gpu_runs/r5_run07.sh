#!/bin/bash
# round 5: the reference recipe (bench.py --recipe, ragged padding-free batches of ~10k tokens) — A/B of the plain
# forward projections on the row-contiguous kernel vs hipBLASLt, and a per-kernel table of the default recipe run
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_07_$n.log 2>&1 || { tail -20 gpurun_out/r5_07_$n.log; exit 1; }
  echo "$n $(grep '"metric"' gpurun_out/r5_07_$n.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["train_pure_samples_per_second"], r["eval_runtime_s"], r["train_runtime_s"])')"
}
for r in 1 2; do
  run base$r X=1
  run fwd$r SFTAMD_TN_CFG=60 SFTAMD_FWD_HIP_N=22016,2048,3072
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof07 -o run -- python bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_07_p.log 2>&1 || { tail -20 gpurun_out/r5_07_p.log; exit 1; }
db=$(ls /tmp/prof07/*/run_results.db /tmp/prof07/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_07_recipe_prof.md > /dev/null
head -30 gpurun_out/r5_07_recipe_prof.md
