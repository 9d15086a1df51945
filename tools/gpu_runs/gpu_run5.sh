#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t5.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t5.log; ok $rc
timeout -k 10 300 python tools/bench_attention.py > gpurun_out/attn5.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/attn5.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b5_mb8.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b5_mb8.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --micro-batch 16 --ga 1 > gpurun_out/b5_mb16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b5_mb16.log; ok $rc
