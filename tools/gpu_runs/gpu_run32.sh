#!/bin/bash
# full GPU tests + bench with fused GEMM epilogues (default) and without (SFTAMD_TN=0) + profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t32.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t32.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b32_tn.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b32_tn.log; [ $rc -eq 0 ] || exit $rc
SFTAMD_TN=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b32_notn.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b32_notn.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/p32.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p32.log
