#!/bin/bash
# Recipe kernel profile + GPU busy timeline (bench.py --recipe, 20 steps, 2 evals): where the per-token gap to the
# synthetic bench goes (kernels vs idle gaps)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof28 -o run -- python -u bench.py --recipe --steps 24 --warmup 0 --eval-steps 1000 > gpurun_out/r3_28_p.log 2>&1 || { tail -20 gpurun_out/r3_28_p.log; exit 1; }
db=$(ls /tmp/prof28/*/run_results.db /tmp/prof28/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r3_28_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 4000 --top 30 --out gpurun_out/r3_28_timeline.md > /dev/null
head -45 gpurun_out/r3_28_prof.md
head -60 gpurun_out/r3_28_timeline.md
grep '"metric"' gpurun_out/r3_28_p.log
