#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
cp tuning/tunableop_results_mi355x.csv gpurun_out/tune_mb16.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_mb16.csv \
  timeout -k 10 900 python bench.py --steps 3 --warmup 2 --micro-batch 16 --ga 1 --tunableop off > gpurun_out/b4_tune16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b4_tune16.log; ok $rc
cp gpurun_out/tune_mb160.csv tuning/tunableop_results_mi355x.csv 2>/dev/null || cp gpurun_out/tune_mb16.csv tuning/tunableop_results_mi355x.csv
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b4_mb8.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b4_mb8.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --micro-batch 16 --ga 1 > gpurun_out/b4_mb16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b4_mb16.log; ok $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python3 bench.py --steps 2 --warmup 2 > gpurun_out/p4.log 2>&1; echo "prof rc=$?" >> gpurun_out/p4.log
ls gpurun_out
