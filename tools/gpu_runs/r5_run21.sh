#!/bin/bash
# full GPU suite after the LoRA / dropout / AdamW / routing changes; LoRA step x2, headline, Llama x2 (shipped selections)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5_21_tests.log 2>&1 || { tail -40 gpurun_out/r5_21_tests.log; exit 1; }
tail -2 gpurun_out/r5_21_tests.log
b() {
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5_21_$n.log 2>&1 || { tail -20 gpurun_out/r5_21_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_21_$n.log | tr '\n' ' ')"
}
b lora1 --freeze-policy lora --steps 20 --warmup 5
b bench1 --steps 20 --warmup 5
b lora2 --freeze-policy lora --steps 20 --warmup 5
b llama1 --model llama3-8b --steps 10 --warmup 3
b llama2 --model llama3-8b --steps 10 --warmup 3
