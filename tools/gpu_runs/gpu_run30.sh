#!/bin/bash
# TN GEMM kernel tests + microbench vs hipBLASLt.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "gemm_tn" --timeout 120 --timeout-method thread > gpurun_out/t30.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t30.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_tn.py > gpurun_out/g30.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/g30.log
