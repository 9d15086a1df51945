#!/bin/bash
# Round 2 baseline: GPU tests, default bench, reference split (8 x GA2), rocprofv3 of the GA2 split.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_01_tests.log 2>&1 || { tail -30 gpurun_out/r2_01_tests.log; exit 1; }
tail -3 gpurun_out/r2_01_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_01_b1.log 2>&1 || { tail -20 gpurun_out/r2_01_b1.log; exit 1; }
grep metric gpurun_out/r2_01_b1.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch 8 --ga 2 > gpurun_out/r2_01_b2.log 2>&1 || { tail -20 gpurun_out/r2_01_b2.log; exit 1; }
grep metric gpurun_out/r2_01_b2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2_01 -o run -- python bench.py --steps 4 --warmup 2 --micro-batch 8 --ga 2 > gpurun_out/r2_01_p.log 2>&1 || { tail -20 gpurun_out/r2_01_p.log; exit 1; }
echo done
