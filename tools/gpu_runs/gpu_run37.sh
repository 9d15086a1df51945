#!/bin/bash
# full GPU test suite + headline bench + rocprofv3 kernel stats of the current default path
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t37.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t37.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b37.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b37.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --optim-state bf16 > gpurun_out/b37_bf16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b37_bf16.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof37 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/p37.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p37.log
