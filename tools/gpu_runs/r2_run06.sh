#!/bin/bash
# Round 2: materialised-dS attention backward: tests, microbench (B=16 x T=512), bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 120 --timeout-method thread > gpurun_out/r2_06_tests.log 2>&1 || { tail -40 gpurun_out/r2_06_tests.log; exit 1; }
tail -1 gpurun_out/r2_06_tests.log
B=16 ATTN_QUICK=1 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/r2_06_attn.log 2>&1 || { tail -20 gpurun_out/r2_06_attn.log; exit 1; }
cat gpurun_out/r2_06_attn.log | grep impl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_06_b.log 2>&1 || { tail -20 gpurun_out/r2_06_b.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/r2_06_b.log
SFTAMD_ATTN_DS_MB=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_06_b0.log 2>&1 || { tail -20 gpurun_out/r2_06_b0.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/r2_06_b0.log
