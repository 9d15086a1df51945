#!/bin/bash
# tn5 variants: one tile per WG (51), K stagger 4/16 (52/53), no-store ablations (54 persistent / 56 per-tile), 55/57
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,51,52,53,54,55,56,57 --plain-only --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048 > gpurun_out/r4_02_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_02_gemm8k.log; exit 1; }
cat gpurun_out/r4_02_gemm8k.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,51,52,53,54,55,56,57 --plain-only --shapes gate_up:22016:2048,lm_head:128256:2048 > gpurun_out/r4_02_gemm8k_b.log 2>&1 || { tail -20 gpurun_out/r4_02_gemm8k_b.log; exit 1; }
cat gpurun_out/r4_02_gemm8k_b.log
