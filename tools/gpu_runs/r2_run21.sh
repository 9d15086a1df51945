#!/bin/bash
# dgrad BK64 default (cfg 7): kernel + model tests, then same-box A/B vs the previous commit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_21_tests.log 2>&1 || { tail -40 gpurun_out/r2_21_tests.log; exit 1; }
tail -1 gpurun_out/r2_21_tests.log
R=3 bash tools/gpu_runs/r2_ab.sh
