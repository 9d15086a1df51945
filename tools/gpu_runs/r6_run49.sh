#!/bin/bash
# round 6: lm_head weight gradient, leftover round split 2 vs 3 vs 4 ways (hybrid)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_ab.py wgrad lm_head,down 1214,1314,1414 --rounds 7 > gpurun_out/r6_49.log 2>&1 || { tail -20 gpurun_out/r6_49.log; exit 1; }
cat gpurun_out/r6_49.log
