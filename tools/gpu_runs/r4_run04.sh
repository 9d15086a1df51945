#!/bin/bash
# tn5 epilogue stores: nt (160), hipBLASLt's 4-row x 256-B pattern (161, timing only), both (162), nt + stagger (163)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,52,54,160,161,162,163 --plain-only --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008 > gpurun_out/r4_04_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_04_gemm8k.log; exit 1; }
cat gpurun_out/r4_04_gemm8k.log
