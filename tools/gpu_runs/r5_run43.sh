#!/bin/bash
# TunableOp selections re-tuned from scratch on this box (forward GEMMs forced onto the library while tuning) vs the shipped file
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/tune_fresh.csv
( while sleep 50; do echo "[tune] still running $(date +%T)"; done ) &
HB=$!
SFTAMD_FWD_GEMM=blas SFTAMD_GEMM_TUNING_FILE=gpurun_out/tune_fresh.csv timeout -k 10 900 python -u bench.py --tunableop tune --steps 2 --warmup 1 > gpurun_out/r5_43_tune.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -20 gpurun_out/r5_43_tune.log; exit 1; }
grep -c "" gpurun_out/tune_fresh.csv
for v in fresh shipped fresh shipped; do
  if [ $v = fresh ]; then f=gpurun_out/tune_fresh.csv; else f=tuning/tunableop_results_mi355x.csv; fi
  SFTAMD_GEMM_TUNING_FILE=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_43_$v.log 2>&1 || { tail -20 gpurun_out/r5_43_$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_43_$v.log | tr '\n' ' ')"
done
