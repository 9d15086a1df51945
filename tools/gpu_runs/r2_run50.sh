#!/bin/bash
# qkv weight gradient on the 2-way split 256x256 ring (cfg 210): wgrad / fused-norm / model tests + bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ddp_gpu.py tests/test_model_gpu.py -k "wgrad or norm or model or zero" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_50_tests.log 2>&1 || { tail -40 gpurun_out/r2_50_tests.log; exit 1; }
tail -1 gpurun_out/r2_50_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_50_b.log 2>&1 || { tail -30 gpurun_out/r2_50_b.log; exit 1; }
  tail -1 gpurun_out/r2_50_b.log | cut -c1-140
done
