#!/bin/bash
# End-of-session: full GPU suite, smoke, default bench, then the reference recipe on its own dataset (r2_run63.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_64_tests.log 2>&1 || { tail -40 gpurun_out/r2_64_tests.log; exit 1; }
tail -1 gpurun_out/r2_64_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_64_smoke.log 2>&1 || { tail -30 gpurun_out/r2_64_smoke.log; exit 1; }
tail -1 gpurun_out/r2_64_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_64_b.log 2>&1 || { tail -30 gpurun_out/r2_64_b.log; exit 1; }
tail -1 gpurun_out/r2_64_b.log | cut -c1-150
tail -1 gpurun_out/r2_64_b.log >> gpurun_out/r2_64_bench.jsonl
bash tools/gpu_runs/r2_run63.sh
