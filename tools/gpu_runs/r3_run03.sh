#!/bin/bash
# 4-wave GEMM schedule variants: FRONT reads (13), split DMA (14), both (15), early barrier (16, 17 = +FRONT, 19 = all)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave" \
  > gpurun_out/r3_03_test.log 2>&1 || { tail -40 gpurun_out/r3_03_test.log; exit 1; }
tail -2 gpurun_out/r3_03_test.log
timeout -k 10 400 python -u tools/bench_gemm_tn.py --cfgs 11,12,13,14,15,16,17,19 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048 > gpurun_out/r3_03.log 2>&1 || { tail -30 gpurun_out/r3_03.log; exit 1; }
cat gpurun_out/r3_03.log
