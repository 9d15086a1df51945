#!/bin/bash
# round 5: dgrad cfg 8 / 9 / 10 (start stagger) for the SwiGLU-backward down dgrad; AdamW SR vs RN bandwidth
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
DGRAD_CFGS=7,8,9,10 DGRAD_SHAPES=swiglu_only timeout -k 10 300 python -u tools/bench_dgrad.py --rounds 4 > gpurun_out/r5_13_dgrad.log 2>&1 || { tail -20 gpurun_out/r5_13_dgrad.log; exit 1; }
grep swiglu gpurun_out/r5_13_dgrad.log | cut -c1-300
timeout -k 10 300 python -u tools/bench_adamw.py > gpurun_out/r5_13_adamw.log 2>&1 || { tail -20 gpurun_out/r5_13_adamw.log; exit 1; }
grep moments gpurun_out/r5_13_adamw.log
