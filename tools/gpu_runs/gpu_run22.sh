#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t22.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t22.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b22_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b22_lora.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b22.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b22.log
