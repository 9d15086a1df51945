#!/bin/bash
# Persistent ping-pong TN GEMM (cfg 12/13): correctness, then bench vs cfg 11 and hipBLASLt.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn_plain" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_26_tests.log 2>&1 || { tail -40 gpurun_out/r2_26_tests.log; exit 1; }
tail -1 gpurun_out/r2_26_tests.log
timeout -k 10 300 python tools/bench_gemm_tn.py --cfgs 11,12,13 --plain-only 2>&1 | tee gpurun_out/r2_26.md
timeout -k 10 300 python tools/bench_gemm_tn.py --cfgs 11,12,13 --plain-only --shapes gu1k:22016:1024,gu4k:22016:4096,sq8k:8192:8192 2>&1 | tee -a gpurun_out/r2_26.md
