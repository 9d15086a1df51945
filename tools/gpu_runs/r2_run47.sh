#!/bin/bash
# Sparse tied-embedding exchange (world > 1 default): full GPU suite (2-ranks-on-one-GPU gloo paths included),
# the 2-rank bench rehearsal on one GPU, smoke, 1-GPU bench (unchanged path).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_47_tests.log 2>&1 || { tail -40 gpurun_out/r2_47_tests.log; exit 1; }
tail -1 gpurun_out/r2_47_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_47_smoke.log 2>&1 || { tail -30 gpurun_out/r2_47_smoke.log; exit 1; }
tail -1 gpurun_out/r2_47_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_47_bench.log 2>&1 || { tail -30 gpurun_out/r2_47_bench.log; exit 1; }
tail -1 gpurun_out/r2_47_bench.log | cut -c1-160
