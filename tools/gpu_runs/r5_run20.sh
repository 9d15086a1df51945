#!/bin/bash
# LoRA: block dxa + wave-private widening — tests, standalone kernels, dxa microbench, LoRA step x2
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
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_20_lora$i.log 2>&1 || { tail -20 gpurun_out/r5_20_lora$i.log; exit 1; }
  echo "lora $(grep -o '"value": [0-9.]*' gpurun_out/r5_20_lora$i.log)"
done
