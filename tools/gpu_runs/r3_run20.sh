#!/bin/bash
# Recipe kernel profile + GPU busy timeline (bench.py --recipe, 20 steps, 2 evals): where the per-token gap to the
# synthetic bench goes (kernels vs idle gaps)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof20 -o run -- python -u bench.py --recipe --steps 20 --warmup 0 > gpurun_out/r3_20_p.log 2>&1 || { tail -20 gpurun_out/r3_20_p.log; exit 1; }
db=$(ls /tmp/prof20/*/run_results.db /tmp/prof20/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r3_20_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 4000 --top 30 --out gpurun_out/r3_20_timeline.md > /dev/null
head -45 gpurun_out/r3_20_prof.md
head -60 gpurun_out/r3_20_timeline.md
grep '"metric"' gpurun_out/r3_20_p.log
