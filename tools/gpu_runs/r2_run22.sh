#!/bin/bash
# Kernel profile of the current default bench step (8 steps incl. warmup), summarised on the box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof22 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r2_22_p.log 2>&1 || { tail -20 gpurun_out/r2_22_p.log; exit 1; }
grep metric gpurun_out/r2_22_p.log
db=$(ls /tmp/prof22/*/run_results.db /tmp/prof22/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r2_22_prof.md && head -50 gpurun_out/r2_22_prof.md
