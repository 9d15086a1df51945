#!/bin/bash
# per-token gap of the recipe: synthetic bench at the recipe's token count (16 x 621, padding-free) vs the recipe
# without evals (timeline of the training steps only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r3_22_$n.log 2>&1 || { tail -20 gpurun_out/r3_22_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_22_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["tokens_per_sec"], d["peak_mem_gb"])')"
}
run s621 --seq 621
run s621ga --seq 621 --micro-batch 8 --ga 2
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 --eval-steps 1000 > gpurun_out/r3_22_rec_noeval.log 2>&1 || { tail -20 gpurun_out/r3_22_rec_noeval.log; exit 1; }
grep '"metric"' gpurun_out/r3_22_rec_noeval.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rec noeval", d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"])'
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof22 -o run -- python -u bench.py --recipe --steps 24 --warmup 0 --eval-steps 1000 > gpurun_out/r3_22_p.log 2>&1 || { tail -20 gpurun_out/r3_22_p.log; exit 1; }
db=$(ls /tmp/prof22/*/run_results.db /tmp/prof22/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 30 --out gpurun_out/r3_22_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 3000 --top 25 --out gpurun_out/r3_22_timeline.md > /dev/null
head -30 gpurun_out/r3_22_prof.md
head -50 gpurun_out/r3_22_timeline.md
