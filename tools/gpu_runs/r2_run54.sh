#!/bin/bash
# ZeRO-1 on GPU tensors with the clip-norm all-reduce through the peer-memory kernel; IPC test again.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_ipc_allreduce_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_54_tests.log 2>&1 || { tail -40 gpurun_out/r2_54_tests.log; exit 1; }
tail -1 gpurun_out/r2_54_tests.log
