#!/bin/bash
# round 5: the new defaults end to end — headline bench x2, recipe x2 (+ kernel table), LoRA, Llama-3-8B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
b() {
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r5_11_$n.log 2>&1 || { tail -20 gpurun_out/r5_11_$n.log; exit 1; }
  echo "$n $(grep '"metric"' gpurun_out/r5_11_$n.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("train_pure_samples_per_second",""), r["ms_per_step"])')"
}
b bench1 --steps 20 --warmup 5
b recipe1 --recipe --steps 40 --warmup 0
b bench2 --steps 20 --warmup 5
b recipe2 --recipe --steps 40 --warmup 0
b lora --steps 20 --warmup 5 --freeze-policy lora
b llama --model llama3-8b --steps 10 --warmup 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof11 -o run -- python bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_11_p.log 2>&1 || { tail -20 gpurun_out/r5_11_p.log; exit 1; }
db=$(ls /tmp/prof11/*/run_results.db /tmp/prof11/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_11_recipe_prof.md > /dev/null
head -20 gpurun_out/r5_11_recipe_prof.md
