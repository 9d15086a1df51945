#!/bin/bash
# RCCL world-1 test with the INFO-log parser assertions; loader change: trainer GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_gpu.py tests/test_trainer_gpu.py > gpurun_out/r5_38_tests.log 2>&1 || { tail -40 gpurun_out/r5_38_tests.log; exit 1; }
tail -2 gpurun_out/r5_38_tests.log
