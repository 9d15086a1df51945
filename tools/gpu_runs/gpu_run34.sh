#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t34.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t34.log; [ $rc -le 1 ] || exit $rc
B=16 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/a34.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/a34.log
