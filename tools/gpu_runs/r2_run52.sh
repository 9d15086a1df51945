#!/bin/bash
# Peer-memory one-shot all-reduce: two ranks sharing one GPU (bounded waits: a hang ends in the error word).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_ipc_allreduce_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r2_52_tests.log 2>&1 || { tail -40 gpurun_out/r2_52_tests.log; exit 1; }
tail -3 gpurun_out/r2_52_tests.log
