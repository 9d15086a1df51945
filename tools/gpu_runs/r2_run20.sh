#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_context_parallel_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_20_tests.log 2>&1 || { tail -40 gpurun_out/r2_20_tests.log; exit 1; }
tail -1 gpurun_out/r2_20_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_20_b$r.log 2>&1 || { tail -20 gpurun_out/r2_20_b$r.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r2_20_b$r.log
done
