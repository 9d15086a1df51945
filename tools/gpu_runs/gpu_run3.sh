#!/bin/bash
# GPU session 3: tests, bench, TunableOp tuning pass.
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t3.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t3.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b3.log 2>&1; rc=$?; echo "bench rc=$rc" >> gpurun_out/b3.log; ok $rc
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 900 python bench.py --steps 5 --warmup 3 --tunableop off > gpurun_out/b3_tune.log 2>&1; rc=$?; echo "tune rc=$rc" >> gpurun_out/b3_tune.log; ok $rc
ls gpurun_out/
