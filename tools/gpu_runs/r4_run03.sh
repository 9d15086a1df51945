#!/bin/bash
# tn5: does desynchronising the workgroups' tile boundaries (start delay, cfg 58 / 59) remove the store stall?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,52,54,58,59 --plain-only --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008 > gpurun_out/r4_03_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_03_gemm8k.log; exit 1; }
cat gpurun_out/r4_03_gemm8k.log
