#!/bin/bash
# Llama-3-8B kernel table (what the 8B step spends its time on at the shipped routing)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof25 -o run -- python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/r5_25_p.log 2>&1 || { tail -20 gpurun_out/r5_25_p.log; exit 1; }
db=$(ls /tmp/prof25/*/run_results.db /tmp/prof25/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r5_25_llama_prof.md > /dev/null
head -44 gpurun_out/r5_25_llama_prof.md
