#!/bin/bash
# round 6: end-of-round kernel tables of the LoRA and Llama-3-8B steps (timed steps only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof70l -o run -- python bench.py --freeze-policy lora --steps 6 --warmup 2 > gpurun_out/r6_70_lora.log 2>&1 || { tail -20 gpurun_out/r6_70_lora.log; exit 1; }
db=$(ls /tmp/prof70l/*/run_results.db /tmp/prof70l/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --window adamw_kernel 2 --title "LoRA step, timed steps only" --out gpurun_out/r6_70_lora.md > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof70b -o run -- python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/r6_70_llama.log 2>&1 || { tail -20 gpurun_out/r6_70_llama.log; exit 1; }
db=$(ls /tmp/prof70b/*/run_results.db /tmp/prof70b/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --window adamw_kernel 4 --title "Llama-3-8B step, timed steps only" --out gpurun_out/r6_70_llama.md > /dev/null
head -12 gpurun_out/r6_70_lora.md; head -12 gpurun_out/r6_70_llama.md
