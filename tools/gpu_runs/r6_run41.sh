#!/bin/bash
# round 6: headline kernel table restricted to the timed steps (window: after the warmup's AdamW launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof41 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_41_ps.log 2>&1 || { tail -20 gpurun_out/r6_41_ps.log; exit 1; }
db=$(ls /tmp/prof41/*/run_results.db /tmp/prof41/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --window adamw_kernel 4 --title "headline step, timed steps only" --out gpurun_out/r6_41_steps.md > /dev/null
python tools/prof_summary.py $db --top 45 --out gpurun_out/r6_41_all.md > /dev/null
head -40 gpurun_out/r6_41_steps.md
