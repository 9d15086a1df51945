#!/bin/bash
# Ping-pong wgrad (cfg 12): correctness, microbench vs the ring kernels and hipBLASLt.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_33_tests.log 2>&1 || { tail -40 gpurun_out/r2_33_tests.log; exit 1; }
tail -1 gpurun_out/r2_33_tests.log
timeout -k 10 300 python tools/bench_wgrad.py --cfgs 10,12,9 2>&1 | tee gpurun_out/r2_33_bench.md
