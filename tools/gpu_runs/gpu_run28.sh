#!/bin/bash
# GPU tests + headline bench (fp32 / bf16 Adam state) + rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t28.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t28.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b28_fp32.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b28_fp32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --optim-state bf16 > gpurun_out/b28_bf16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b28_bf16.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof28 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/p28.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p28.log
