#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t8.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t8.log; ok $rc
timeout -k 10 500 python bench.py --steps 4 --warmup 2 --model llama3-8b > gpurun_out/b8_llama.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b8_llama.log; ok $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b8_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b8_lora.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-master-weights > gpurun_out/b8_nomaster.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b8_nomaster.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b8.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b8.log; ok $rc
