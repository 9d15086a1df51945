#!/bin/bash
# end-of-round validation: full GPU suite, smoke, headline x2, LoRA x2, Llama-3-8B, recipe (HF + pure)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5_35_tests.log 2>&1 || { tail -40 gpurun_out/r5_35_tests.log; exit 1; }
tail -2 gpurun_out/r5_35_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_35_smoke.log 2>&1 || { tail -20 gpurun_out/r5_35_smoke.log; exit 1; }
tail -1 gpurun_out/r5_35_smoke.log
b() {
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r5_35_$n.log 2>&1 || { tail -20 gpurun_out/r5_35_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*\|"loss_finite": [a-z]*' gpurun_out/r5_35_$n.log | tr '\n' ' ')"
}
b bench1 --steps 20 --warmup 5
b lora1 --freeze-policy lora --steps 20 --warmup 5
b bench2 --steps 20 --warmup 5
b lora2 --freeze-policy lora --steps 20 --warmup 5
b llama1 --model llama3-8b --steps 10 --warmup 3
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_35_recipe.log 2>&1 || { tail -20 gpurun_out/r5_35_recipe.log; exit 1; }
echo "recipe $(grep '"metric"' gpurun_out/r5_35_recipe.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("train_pure_samples_per_second",""), r.get("final_loss", ""))')"
