#!/bin/bash
# Attention forward ablation (where the 48 us go) + per-shape GEMM audit of the current default step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/attn_ablate.py > gpurun_out/r2_42_ablate.log 2>&1 || { tail -20 gpurun_out/r2_42_ablate.log; exit 1; }
grep DIAG gpurun_out/r2_42_ablate.log
timeout -k 10 300 python tools/gemm_audit.py > gpurun_out/r2_42_gemm_audit.txt 2>&1 || { tail -20 gpurun_out/r2_42_gemm_audit.txt; exit 1; }
grep -v Warning gpurun_out/r2_42_gemm_audit.txt | tail -40
