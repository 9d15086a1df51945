#!/bin/bash
# fwd32 + dkdv32 (32x32x16 attention): numerics vs fp32, every attention test, microbench vs fwd3 / dkdv5; dgrad bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_fwd_out_and_lse or smollm3_shape" > gpurun_out/r4_13_fwd.log 2>&1 || { tail -40 gpurun_out/r4_13_fwd.log; exit 1; }
tail -3 gpurun_out/r4_13_fwd.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or flash or attn" > gpurun_out/r4_13_attn.log 2>&1 || { tail -40 gpurun_out/r4_13_attn.log; exit 1; }
tail -2 gpurun_out/r4_13_attn.log
B=16 timeout -k 10 300 python -u tools/bench_attention.py > gpurun_out/r4_13_bench.log 2>&1 || { tail -20 gpurun_out/r4_13_bench.log; exit 1; }
cat gpurun_out/r4_13_bench.log
DGRAD_CFGS=7,13 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r4_13_dgrad.log 2>&1 || { tail -20 gpurun_out/r4_13_dgrad.log; exit 1; }
grep shape gpurun_out/r4_13_dgrad.log
