#!/bin/bash
# Llama-3-8B: TunableOp selections for its forward projections (hipBLASLt), then the forward routing A/B
# (auto: hipBLASLt for the now-tuned shapes, hip: the row-contiguous persistent kernel everywhere)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cp tuning/tunableop_results_mi355x.csv gpurun_out/tune_llama.csv
( while sleep 50; do echo "[tune] still tuning $(date +%T)"; done ) &
HB=$!
SFTAMD_FWD_GEMM=blas SFTAMD_GEMM_TUNING_FILE=gpurun_out/tune_llama.csv timeout -k 10 900 python -u bench.py --model llama3-8b --steps 2 --warmup 1 --tunableop tune > gpurun_out/r5_17_tune.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -20 gpurun_out/r5_17_tune.log; exit 1; }
grep -c "" gpurun_out/tune_llama.csv
for arm in auto hip auto hip; do
  SFTAMD_FWD_GEMM=$arm SFTAMD_GEMM_TUNING_FILE=gpurun_out/tune_llama.csv timeout -k 10 200 python -u bench.py --model llama3-8b --steps 10 --warmup 3 > gpurun_out/r5_17_$arm.log 2>&1 || { tail -20 gpurun_out/r5_17_$arm.log; exit 1; }
  echo "llama $arm $(grep -o '"value": [0-9.]*' gpurun_out/r5_17_$arm.log)"
done
