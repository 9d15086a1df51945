#!/bin/bash
# Context-parallel building blocks on the HIP kernels + full GPU suite.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t58.log 2>&1 || { tail -40 gpurun_out/t58.log; exit 1; }
tail -2 gpurun_out/t58.log
