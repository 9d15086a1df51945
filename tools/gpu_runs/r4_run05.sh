#!/bin/bash
# pruned attention (default + dq3 fallback only): GPU tests + microbench; tn5 epilogue store experiments
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > gpurun_out/r4_05_attn_tests.log 2>&1 || { tail -30 gpurun_out/r4_05_attn_tests.log; exit 1; }
tail -2 gpurun_out/r4_05_attn_tests.log
timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r4_05_attn_bench.log 2>&1 || { tail -20 gpurun_out/r4_05_attn_bench.log; exit 1; }
cat gpurun_out/r4_05_attn_bench.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,52,54,160,161,162,163 --plain-only --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008 > gpurun_out/r4_05_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_05_gemm8k.log; exit 1; }
cat gpurun_out/r4_05_gemm8k.log
