#!/bin/bash
# LoRA widening prefetch depth 1 / 2 / 3: tests, standalone, LoRA step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2 3; do
  SFTAMD_LORA_TSUM_PD=$v SFTAMD_LORA_FWD_PD=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora_fwd_bwd" > gpurun_out/r5_22_tests$v.log 2>&1 || { tail -30 gpurun_out/r5_22_tests$v.log; exit 1; }
  tail -1 gpurun_out/r5_22_tests$v.log
done
timeout -k 10 200 python -u tools/bench_lora_kernels.py > gpurun_out/r5_22_kern.log 2>&1 || { tail -20 gpurun_out/r5_22_kern.log; exit 1; }
grep "pd\|swiglu\|tsum" gpurun_out/r5_22_kern.log
for v in 2 1 3 2 1 3; do
  SFTAMD_LORA_FWD_PD=$v timeout -k 10 300 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_22_lora$v.log 2>&1 || { tail -20 gpurun_out/r5_22_lora$v.log; exit 1; }
  echo "lora pd$v $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_22_lora$v.log | tr '\n' ' ')"
done
# recipe: gate_up + SwiGLU fused by default for the untuned (ragged) shapes vs the plain kernel + SwiGLU pass
for v in 1 0 1 0; do
  SFTAMD_GU_AUTO=$v timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_22_recipe$v.log 2>&1 || { tail -20 gpurun_out/r5_22_recipe$v.log; exit 1; }
  echo "recipe gu_auto$v $(grep '"metric"' gpurun_out/r5_22_recipe$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("train_pure_samples_per_second",""), r.get("final_loss", ""))')"
done
