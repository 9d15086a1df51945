#!/bin/bash
# Ragged real-data shapes (16 x 640 tokens, M = 10240): does a TunableOp selection for the M = 10240 GEMMs beat the
# library default heuristics the shipped file falls back to? bench --seq 640 before / after tuning, interleaved.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 bash tools/tune_gemms.sh gpurun_out/tune640.csv --seq 640 > gpurun_out/r2_65_tune.log 2>&1 || { tail -30 gpurun_out/r2_65_tune.log; exit 1; }
T=gpurun_out/tune6400.csv; [ -f $T ] || T=gpurun_out/tune640.csv
echo "tuned file $T: $(wc -l < $T) lines"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seq 640 > gpurun_out/r2_65_base.log 2>&1 || { tail -30 gpurun_out/r2_65_base.log; exit 1; }
  echo "shipped file: $(tail -1 gpurun_out/r2_65_base.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  SFTAMD_GEMM_TUNING_FILE=$T timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seq 640 > gpurun_out/r2_65_tuned.log 2>&1 || { tail -30 gpurun_out/r2_65_tuned.log; exit 1; }
  echo "tuned file:   $(tail -1 gpurun_out/r2_65_tuned.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
