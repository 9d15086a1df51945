#!/bin/bash
# Diagnostics: pure fwd+bwd time (no optimizer), optimizer overlap on/off, attention microbench at B=16.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=tuning/tunableop_results_mi355x.csv
timeout -k 10 300 python tools/quick_step.py --batch 16 --steps 6 > gpurun_out/q29.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/q29.log; [ $rc -eq 0 ] || exit $rc
unset PYTORCH_TUNABLEOP_ENABLED PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_FILENAME
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --optim-state bf16 --no-overlap > gpurun_out/b29_nooverlap.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b29_nooverlap.log; [ $rc -eq 0 ] || exit $rc
B=16 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/a29.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/a29.log
