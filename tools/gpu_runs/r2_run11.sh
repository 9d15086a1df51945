#!/bin/bash
# Round 2: per-shape GEMM audit of the current default step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python tools/gemm_audit.py > gpurun_out/r2_11_gemm_audit.txt 2>&1 || { tail -20 gpurun_out/r2_11_gemm_audit.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_11_gemm_audit.txt | head -40
