#!/bin/bash
# Checkpoint: full GPU suite, smoke, default bench (x2), reference split.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_55_tests.log 2>&1 || { tail -40 gpurun_out/r2_55_tests.log; exit 1; }
tail -1 gpurun_out/r2_55_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_55_smoke.log 2>&1 || { tail -30 gpurun_out/r2_55_smoke.log; exit 1; }
tail -1 gpurun_out/r2_55_smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_55_b.log 2>&1 || { tail -30 gpurun_out/r2_55_b.log; exit 1; }
  tail -1 gpurun_out/r2_55_b.log | cut -c1-150
  tail -1 gpurun_out/r2_55_b.log >> gpurun_out/r2_55_bench.jsonl
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch 8 --ga 2 > gpurun_out/r2_55_ga2.log 2>&1 || { tail -30 gpurun_out/r2_55_ga2.log; exit 1; }
tail -1 gpurun_out/r2_55_ga2.log | cut -c1-150
tail -1 gpurun_out/r2_55_ga2.log >> gpurun_out/r2_55_bench.jsonl
