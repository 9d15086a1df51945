#!/bin/bash
# LoRA adapter-dx on MFMA vs the LDS/VALU kernel (standalone + in-step A/B); AdamW UNR 4 vs 2 in the training step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k lora > gpurun_out/r5_16_tests.log 2>&1 || { tail -30 gpurun_out/r5_16_tests.log; exit 1; }
tail -2 gpurun_out/r5_16_tests.log
timeout -k 10 200 python -u tools/bench_lora_kernels.py > gpurun_out/r5_16_kern.log 2>&1 || { tail -20 gpurun_out/r5_16_kern.log; exit 1; }
cat gpurun_out/r5_16_kern.log | grep -v amdgpu.ids
for v in 1 0 1 0; do
  SFTAMD_LORA_DX=$v timeout -k 10 200 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_16_lora_$v.log 2>&1 || { tail -20 gpurun_out/r5_16_lora_$v.log; exit 1; }
  echo "lora dx$v $(grep -o '"value": [0-9.]*' gpurun_out/r5_16_lora_$v.log)"
done
for u in 4 2 4 2; do
  SFTAMD_ADAMW_UNR=$u timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_16_unr$u.log 2>&1 || { tail -20 gpurun_out/r5_16_unr$u.log; exit 1; }
  echo "headline unr$u $(grep -o '"value": [0-9.]*' gpurun_out/r5_16_unr$u.log)"
done
for wg in 768 512 1024 768 512 1024; do
  SFTAMD_LORA_TSUM_WG=$wg timeout -k 10 200 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_16_tsum$wg.log 2>&1 || { tail -20 gpurun_out/r5_16_tsum$wg.log; exit 1; }
  echo "lora tsum_wg$wg $(grep -o '"value": [0-9.]*' gpurun_out/r5_16_tsum$wg.log)"
done
