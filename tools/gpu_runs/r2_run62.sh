#!/bin/bash
# End-of-session step profile of the default path: rocprofv3 kernel summary + GPU busy timeline, and the 8 x GA 2
# reference split's kernel summary.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof62 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r2_62_p.log 2>&1 || { tail -20 gpurun_out/r2_62_p.log; exit 1; }
db=$(ls /tmp/prof62/*/run_results.db /tmp/prof62/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r2_62_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 600 --top 20 --out gpurun_out/r2_62_timeline.md > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof62g -o run -- python bench.py --steps 6 --warmup 2 --micro-batch 8 --ga 2 > gpurun_out/r2_62_pg.log 2>&1 || { tail -20 gpurun_out/r2_62_pg.log; exit 1; }
db=$(ls /tmp/prof62g/*/run_results.db /tmp/prof62g/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r2_62_prof_ga2.md > /dev/null
head -30 gpurun_out/r2_62_prof.md
head -12 gpurun_out/r2_62_timeline.md
