#!/bin/bash
# attention v6 forward (r3_run10) + chunked LM head test, then the persistent GEMM + forward-routing A/B (r3_run09)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_runs/r3_run10.sh || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lm_head_chunked_gpu.py \
  > gpurun_out/r3_12_lmhead.log 2>&1 || { tail -30 gpurun_out/r3_12_lmhead.log; exit 1; }
tail -2 gpurun_out/r3_12_lmhead.log
bash tools/gpu_runs/r3_run09.sh
