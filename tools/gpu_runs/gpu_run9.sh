#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "flash or adamw" > gpurun_out/t9.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t9.log; ok $rc
timeout -k 10 300 python tools/bench_attention.py > gpurun_out/attn9.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/attn9.log; ok $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b9_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b9_lora.log; ok $rc
