#!/bin/bash
# End-of-session checkpoint: full GPU suite, default bench, kernel profile + timeline, recipe
# (parquet + evals every 10 steps) through bench.py --recipe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r3_48_tests.log 2>&1 || { tail -40 gpurun_out/r3_48_tests.log; exit 1; }
tail -2 gpurun_out/r3_48_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_48_bench.log 2>&1 || { tail -20 gpurun_out/r3_48_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_48_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof48 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r3_48_p.log 2>&1 || { tail -20 gpurun_out/r3_48_p.log; exit 1; }
db=$(ls /tmp/prof48/*/run_results.db /tmp/prof48/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r3_48_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 600 --top 20 --out gpurun_out/r3_48_timeline.md > /dev/null
head -30 gpurun_out/r3_48_prof.md
timeout -k 10 600 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_48_recipe.log 2>&1 || { tail -30 gpurun_out/r3_48_recipe.log; exit 1; }
grep '"metric"' gpurun_out/r3_48_recipe.log
