#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_generation_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/t35.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t35.log
