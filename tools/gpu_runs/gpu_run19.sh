#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t19.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t19.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b19.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b19.log; [ $rc -eq 0 ] || exit $rc
SFTAMD_WGRAD=blas timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b19_blas.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b19_blas.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o run -- python bench.py --steps 5 --warmup 2 --no-overlap > gpurun_out/p19.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p19.log
