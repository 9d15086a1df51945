#!/bin/bash
# LoRA kernel tests after the cleanup (MFMA dx only, one-launch scatters), then the headline per-op attribution
# (r5_run18) and the Llama-3-8B TunableOp tuning + forward routing A/B (r5_run17)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py -k "lora or adamw" > gpurun_out/r5_19_tests.log 2>&1 || { tail -30 gpurun_out/r5_19_tests.log; exit 1; }
tail -1 gpurun_out/r5_19_tests.log
bash tools/gpu_runs/r5_run18.sh && bash tools/gpu_runs/r5_run17.sh
