#!/bin/bash
# Checkpoint of the session's default path: full GPU suite, smoke, bench, step kernel profile + timeline, copy audit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_39_tests.log 2>&1 || { tail -40 gpurun_out/r2_39_tests.log; exit 1; }
tail -1 gpurun_out/r2_39_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_39_smoke.log 2>&1 || { tail -30 gpurun_out/r2_39_smoke.log; exit 1; }
tail -1 gpurun_out/r2_39_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_39_bench.log 2>&1 || { tail -30 gpurun_out/r2_39_bench.log; exit 1; }
tail -1 gpurun_out/r2_39_bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof39 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r2_39_p.log 2>&1 || { tail -20 gpurun_out/r2_39_p.log; exit 1; }
db=$(ls /tmp/prof39/*/run_results.db /tmp/prof39/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r2_39_prof.md > /dev/null
python tools/prof_timeline.py $db --window-ms 600 --top 20 --out gpurun_out/r2_39_timeline.md > /dev/null
timeout -k 10 300 python tools/copy_audit.py > gpurun_out/r2_39_copy_audit.txt 2>&1 || { tail -20 gpurun_out/r2_39_copy_audit.txt; exit 1; }
head -3 gpurun_out/r2_39_copy_audit.txt
