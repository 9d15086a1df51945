#!/bin/bash
# round 6: headline kernel table of the timed steps after the paired weight gradients
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof48 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_48_ps.log 2>&1 || { tail -20 gpurun_out/r6_48_ps.log; exit 1; }
db=$(ls /tmp/prof48/*/run_results.db /tmp/prof48/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --window adamw_kernel 4 --title "headline step, timed steps only" --out gpurun_out/r6_48_steps.md > /dev/null
python tools/prof_summary.py $db --top 45 --out gpurun_out/r6_48_all.md > /dev/null
head -40 gpurun_out/r6_48_steps.md
