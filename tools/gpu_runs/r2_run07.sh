#!/bin/bash
# Round 2: per-kernel times of the v4 attention backward (rocprofv3 over the attention microbench).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=16 ATTN_QUICK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2_07 -o run -- python tools/bench_attention.py > gpurun_out/r2_07.log 2>&1 || { tail -20 gpurun_out/r2_07.log; exit 1; }
grep impl gpurun_out/r2_07.log
