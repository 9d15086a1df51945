#!/bin/bash
# Per-shape GEMM efficiency inside one training step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_audit.py > gpurun_out/gemm_audit53.txt 2>&1 || { tail -20 gpurun_out/gemm_audit53.txt; exit 1; }
grep -v Warning gpurun_out/gemm_audit53.txt | tail -40
