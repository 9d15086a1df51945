#!/bin/bash
# LoRA adapter-dx pass: MFMA (no LDS) vs the LDS/VALU kernel — numerics tests, standalone timings, LoRA bench A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora" tests/test_model_gpu.py -k "lora" > gpurun_out/r5_15_tests.log 2>&1 \
  && timeout -k 10 200 python -u tools/bench_lora_kernels.py > gpurun_out/r5_15_kern.log 2>&1 \
  && for v in 1 0 1 0; do SFTAMD_LORA_DX=$v timeout -k 10 200 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_15_lora_$v.log 2>&1 || exit 1; grep -o '"value": [0-9.]*' gpurun_out/r5_15_lora_$v.log | sed "s/^/dx$v /"; done
rc=$?
tail -3 gpurun_out/r5_15_tests.log; cat gpurun_out/r5_15_kern.log
exit $rc
