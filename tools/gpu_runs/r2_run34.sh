#!/bin/bash
# Re-entry check: full GPU suite, smoke, default 1-GPU bench, reference split (8 x GA2).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_34_tests.log 2>&1 || { tail -40 gpurun_out/r2_34_tests.log; exit 1; }
tail -2 gpurun_out/r2_34_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_34_smoke.log 2>&1 || { tail -30 gpurun_out/r2_34_smoke.log; exit 1; }
tail -1 gpurun_out/r2_34_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r2_34_bench.log 2>&1 || { tail -30 gpurun_out/r2_34_bench.log; exit 1; }
tail -1 gpurun_out/r2_34_bench.log
timeout -k 10 400 python bench.py --micro-batch 8 --ga 2 > gpurun_out/r2_34_bench_ga2.log 2>&1 || { tail -30 gpurun_out/r2_34_bench_ga2.log; exit 1; }
tail -1 gpurun_out/r2_34_bench_ga2.log
