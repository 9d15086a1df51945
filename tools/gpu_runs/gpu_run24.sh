#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --freeze-policy lora --tunableop tune > gpurun_out/tune24.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/tune24.log; cp tuning/tunableop_results_mi355x.csv gpurun_out/tuned24.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b24_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b24_lora.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof24_lora -o run -- python bench.py --steps 4 --warmup 2 --freeze-policy lora --no-overlap > gpurun_out/p24_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p24_lora.log
