#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b27_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b27_lora.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof27_lora -o run -- python bench.py --steps 4 --warmup 2 --freeze-policy lora --no-overlap > gpurun_out/p27_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p27_lora.log
