#!/bin/bash
# LoRA: block dxa, wave-private widening, paired-hash dropout, wave-private wide tsum (A/B) — tests, standalone
# kernels, dxa microbench, LoRA step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "lora or dropout" > gpurun_out/r5_20_tests.log 2>&1 || { tail -30 gpurun_out/r5_20_tests.log; exit 1; }
tail -1 gpurun_out/r5_20_tests.log
timeout -k 10 200 python -u tools/bench_lora_kernels.py > gpurun_out/r5_20_kern.log 2>&1 || { tail -20 gpurun_out/r5_20_kern.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_20_kern.log
timeout -k 10 200 python -u tools/bench_lora_dxa.py > gpurun_out/r5_20_dxa.log 2>&1 || { tail -20 gpurun_out/r5_20_dxa.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_20_dxa.log
timeout -k 10 600 python -u tools/nan_hunt.py --model llama3-8b --reps 5 > gpurun_out/r5_20_nan.log 2>&1 || { tail -20 gpurun_out/r5_20_nan.log; exit 1; }
grep "^rep" gpurun_out/r5_20_nan.log | grep -E "step 13|NON-FINITE|step 1:"
for v in 1 0 1 0; do
  SFTAMD_LORA_TSUM_WP=$v timeout -k 10 200 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_20_lora$v.log 2>&1 || { tail -20 gpurun_out/r5_20_lora$v.log; exit 1; }
  echo "lora wp$v $(grep -o '"value": [0-9.]*' gpurun_out/r5_20_lora$v.log)"
done
