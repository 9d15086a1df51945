#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t26.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t26.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/lora_tune0.csv /tmp/lt.csv 2>/dev/null
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=/tmp/lt.csv timeout -k 10 900 python bench.py --steps 2 --warmup 1 --freeze-policy lora --tunableop off > gpurun_out/tune26.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/tune26.log; ls /tmp/lt*; cp /tmp/lt0.csv gpurun_out/lora_tune26.csv; [ $rc -eq 0 ] || exit $rc
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/lora_tune26.csv timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora --tunableop off > gpurun_out/b26_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b26_lora.log
