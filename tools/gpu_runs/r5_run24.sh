#!/bin/bash
# round-5 validation of the committed tree: full GPU suite, smoke(), headline x2, LoRA, recipe, Llama-3-8B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5_24_tests.log 2>&1 || { tail -40 gpurun_out/r5_24_tests.log; exit 1; }
tail -1 gpurun_out/r5_24_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_24_smoke.log 2>&1 || { tail -20 gpurun_out/r5_24_smoke.log; exit 1; }
tail -1 gpurun_out/r5_24_smoke.log
b() {
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r5_24_$n.log 2>&1 || { tail -20 gpurun_out/r5_24_$n.log; exit 1; }
  echo "$n $(grep '"metric"' gpurun_out/r5_24_$n.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("train_pure_samples_per_second",""), r["ms_per_step"], r.get("final_loss"), r.get("loss_finite"))')"
}
b bench1
b lora --freeze-policy lora --steps 20 --warmup 5
b bench2 --steps 20 --warmup 5
b recipe --recipe --steps 40 --warmup 0
b llama --model llama3-8b --steps 10 --warmup 3
