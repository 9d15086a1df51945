#!/bin/bash
# RCCL world-1 process-group test (high-priority streams, side-stream in-place RS/AG, async count),
# the full GPU suite, and a 1-GPU bench on the current tree.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t63a.log 2>&1 || { tail -40 gpurun_out/t63a.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/t63a.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t63.log 2>&1 || { tail -30 gpurun_out/t63.log; exit 1; }
tail -1 gpurun_out/t63.log
timeout -k 10 300 python bench.py > gpurun_out/b63.log 2>&1 || { tail -20 gpurun_out/b63.log; exit 1; }
grep metric gpurun_out/b63.log
