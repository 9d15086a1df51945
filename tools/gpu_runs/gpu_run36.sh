#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/t36.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t36.log
