#!/bin/bash
# round 6: after the conflict-free dgrad rings — plain input gradients, 4-wave ring (14) vs 8-wave rings (5, 7)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_ab.py dgrad o,qkv,gate_up,down,lm_head 14,5,7 --rounds 7 > gpurun_out/r6_53.log 2>&1 || { tail -20 gpurun_out/r6_53.log; exit 1; }
cat gpurun_out/r6_53.log
