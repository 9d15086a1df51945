#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/attn_ab.py > gpurun_out/r4_16_ab.log 2>&1 || { tail -20 gpurun_out/r4_16_ab.log; exit 1; }
cat gpurun_out/r4_16_ab.log
