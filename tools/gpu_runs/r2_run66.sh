#!/bin/bash
# A/B of the M = 10240 (16 x 640) selections tuned in r2_run65 (tuning/candidate_640.csv = shipped + 5 forward shapes)
# against the shipped file (library defaults for those shapes): bench --seq 640, interleaved.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seq 640 > gpurun_out/r2_66_base.log 2>&1 || { tail -30 gpurun_out/r2_66_base.log; exit 1; }
  echo "shipped file: $(tail -1 gpurun_out/r2_66_base.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  SFTAMD_GEMM_TUNING_FILE=tuning/candidate_640.csv timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seq 640 > gpurun_out/r2_66_tuned.log 2>&1 || { tail -30 gpurun_out/r2_66_tuned.log; exit 1; }
  echo "tuned file:   $(tail -1 gpurun_out/r2_66_tuned.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
