#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t42.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t42.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b42.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b42.log
