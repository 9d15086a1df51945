#!/bin/bash
# 4-wave kernel of gemm_4w.hip on the forward layout (gemm_tn cfg 60 ring / 61 pair) vs cfg 12 / 50 / hipBLASLt
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave" \
  > gpurun_out/r3_15_test.log 2>&1 || { tail -40 gpurun_out/r3_15_test.log; exit 1; }
tail -2 gpurun_out/r3_15_test.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 12,50,60,61 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048 > gpurun_out/r3_15.log 2>&1 || { tail -30 gpurun_out/r3_15.log; exit 1; }
cat gpurun_out/r3_15.log
