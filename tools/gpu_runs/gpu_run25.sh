#!/bin/bash
cd $GRAFT_REPO_ROOT
cp tuning/tunableop_results_mi355x.csv gpurun_out/lora_tune.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/lora_tune.csv timeout -k 10 900 python tools/bench_lora.py > gpurun_out/bl25.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bl25.log
ls gpurun_out/ | grep lora_tune
