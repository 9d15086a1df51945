#!/bin/bash
# round 6: kernel table + timeline (GPU busy) of the headline step after the routing / AdamW changes (serial update)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof13 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_13_ps.log 2>&1 || { tail -20 gpurun_out/r6_13_ps.log; exit 1; }
db=$(ls /tmp/prof13/*/run_results.db /tmp/prof13/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 50 --out gpurun_out/r6_13_step_prof.md > /dev/null
head -50 gpurun_out/r6_13_step_prof.md
python tools/prof_timeline.py $db > gpurun_out/r6_13_timeline.txt 2>&1 || true
tail -30 gpurun_out/r6_13_timeline.txt
