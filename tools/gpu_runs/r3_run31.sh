#!/bin/bash
# persistent forward GEMM (cfg 50) with buffer-descriptor LDS-DMA: tests, microbench vs hipBLASLt, then the
# fused-gate_up / optimizer-overlap A/B (r3_run30)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn" \
  > gpurun_out/r3_31_test.log 2>&1 || { tail -40 gpurun_out/r3_31_test.log; exit 1; }
tail -2 gpurun_out/r3_31_test.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 12,50 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048 > gpurun_out/r3_31.log 2>&1 || { tail -30 gpurun_out/r3_31.log; exit 1; }
cat gpurun_out/r3_31.log
timeout -k 10 200 python -u tools/bench_gemm_tn.py --fused-cfgs 11,50 --iters 30 > gpurun_out/r3_31f.log 2>&1 || { tail -30 gpurun_out/r3_31f.log; exit 1; }
cat gpurun_out/r3_31f.log
bash tools/gpu_runs/r3_run30.sh
