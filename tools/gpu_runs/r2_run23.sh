#!/bin/bash
# Ping-pong TN GEMM (cfg 8/9): correctness then microbench vs hipBLASLt and the BK64 ring.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn_plain" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_23_tests.log 2>&1 || { tail -40 gpurun_out/r2_23_tests.log; exit 1; }
tail -1 gpurun_out/r2_23_tests.log
timeout -k 10 300 python tools/bench_gemm_tn.py --cfgs 5,8,9,10,11 --plain-only 2>&1 | tee gpurun_out/r2_23_bench.md
