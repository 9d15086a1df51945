#!/bin/bash
# round 6: GEMM grids under held CUs (stand-in for RCCL channel blocks overlapped with the backward at N > 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_cu_contention.py --held 0,4,8,16,32 > gpurun_out/r6_32_cu.log 2>&1 || { tail -20 gpurun_out/r6_32_cu.log; exit 1; }
cat gpurun_out/r6_32_cu.log
