#!/bin/bash
# round 6: forward projections, hipBLASLt vs the ping-pong tn3 (cfg 11, the qkv+RoPE kernel without the RoPE) and tn6
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_ab.py fwd qkv,o,gate_up,down,lm_head blas,11,2,60 --rounds 7 > gpurun_out/r6_30_ab.log 2>&1 || { tail -20 gpurun_out/r6_30_ab.log; exit 1; }
cat gpurun_out/r6_30_ab.log
