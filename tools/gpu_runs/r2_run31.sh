#!/bin/bash
# Full GPU suite + smoke + default bench (round-2 state check).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_31_tests.log 2>&1 || { tail -40 gpurun_out/r2_31_tests.log; exit 1; }
tail -2 gpurun_out/r2_31_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2_31_smoke.log 2>&1 || { tail -20 gpurun_out/r2_31_smoke.log; exit 1; }
tail -1 gpurun_out/r2_31_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2_31_bench.log 2>&1 || { tail -20 gpurun_out/r2_31_bench.log; exit 1; }
grep metric gpurun_out/r2_31_bench.log
timeout -k 10 300 python bench.py --micro-batch 8 --ga 2 > gpurun_out/r2_31_bench_ga2.log 2>&1 || { tail -20 gpurun_out/r2_31_bench_ga2.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r2_31_bench_ga2.log
