#!/bin/bash
# Step kernel profile + GPU idle-gap timeline of bench.py (GQA-grouped attention backward default).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof36 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r2_36_p.log 2>&1 || { tail -20 gpurun_out/r2_36_p.log; exit 1; }
db=$(ls /tmp/prof36/*/run_results.db /tmp/prof36/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r2_36_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 600 --top 30 --out gpurun_out/r2_36_timeline.md
