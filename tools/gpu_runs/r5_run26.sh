#!/bin/bash
# LoRA wide forward GEMMs: TunableOp selections for the widened shapes (hipBLASLt / rocBLAS), then the routing A/B
# (auto: the library for the now-tuned shapes; hip: the row-contiguous persistent kernel for all)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py -k "lora" > gpurun_out/r5_26_tests.log 2>&1 || { tail -30 gpurun_out/r5_26_tests.log; exit 1; }
tail -1 gpurun_out/r5_26_tests.log
cp tuning/tunableop_results_mi355x.csv gpurun_out/tune_lora.csv
( while sleep 50; do echo "[tune] still tuning $(date +%T)"; done ) &
HB=$!
SFTAMD_FWD_GEMM=blas SFTAMD_GEMM_TUNING_FILE=gpurun_out/tune_lora.csv timeout -k 10 900 python -u bench.py --freeze-policy lora --steps 2 --warmup 1 --tunableop tune > gpurun_out/r5_26_tune.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -20 gpurun_out/r5_26_tune.log; exit 1; }
grep -c "" gpurun_out/tune_lora.csv
for arm in auto hip auto hip; do
  SFTAMD_FWD_GEMM=$arm SFTAMD_GEMM_TUNING_FILE=gpurun_out/tune_lora.csv timeout -k 10 300 python -u bench.py --freeze-policy lora --steps 20 --warmup 5 > gpurun_out/r5_26_$arm.log 2>&1 || { tail -20 gpurun_out/r5_26_$arm.log; exit 1; }
  echo "lora $arm $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_26_$arm.log | tr '\n' ' ')"
done
