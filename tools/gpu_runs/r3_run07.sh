#!/bin/bash
# persistent 4-wave GEMM (cfg 50): correctness, then timing vs hipBLASLt / cfg 11 / cfg 12 and a K sweep (fixed vs
# per-K cost), plus the cfg 12 epilogue / prologue ablations (1208 no epilogue, 1216 no prologue wait)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave" \
  > gpurun_out/r3_07_test.log 2>&1 || { tail -40 gpurun_out/r3_07_test.log; exit 1; }
tail -2 gpurun_out/r3_07_test.log
timeout -k 10 400 python -u tools/bench_gemm_tn.py --cfgs 11,12,50,1208,1216 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048,gu1k:22016:1024,gu4k:22016:4096,gu8k:22016:8192 > gpurun_out/r3_07.log 2>&1 || { tail -30 gpurun_out/r3_07.log; exit 1; }
cat gpurun_out/r3_07.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 11,12,50 --plain-only --iters 30 --m 10240 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048 > gpurun_out/r3_07b.log 2>&1 || { tail -30 gpurun_out/r3_07b.log; exit 1; }
cat gpurun_out/r3_07b.log
