#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t38.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t38.log; [ $rc -le 1 ] || exit $rc
: > gpurun_out/b38.log
for ws in 1 0 1 0; do
  echo "WGRAD_STREAM=$ws" >> gpurun_out/b38.log
  SFTAMD_WGRAD_STREAM=$ws timeout -k 10 300 python bench.py 2>&1 | grep metric >> gpurun_out/b38.log || exit 1
done
