#!/bin/bash
# full GPU suite + headline bench + LoRA bench after the LoRA SwiGLU fusion and the batched adapter sync
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4_26_tests.log 2>&1 || { tail -40 gpurun_out/r4_26_tests.log; exit 1; }
tail -2 gpurun_out/r4_26_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_26_bench.log 2>&1 || { tail -20 gpurun_out/r4_26_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_26_bench.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_26_lora.log 2>&1 || { tail -20 gpurun_out/r4_26_lora.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_26_lora.log
