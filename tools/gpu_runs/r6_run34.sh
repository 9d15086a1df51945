#!/bin/bash
# round 6: CU-budget-aware 4-wave grids under held CUs (RCCL stand-in): headline step, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_34.log; : > $out
timeout -k 10 300 python -u tools/bench_cu_contention.py --held 0,8 > gpurun_out/r6_34_cu_b256.log 2>&1 || { tail -20 gpurun_out/r6_34_cu_b256.log; exit 1; }
SFTAMD_CU_BUDGET=248 timeout -k 10 300 python -u tools/bench_cu_contention.py --held 0,8 > gpurun_out/r6_34_cu_b248.log 2>&1 || { tail -20 gpurun_out/r6_34_cu_b248.log; exit 1; }
for cfg in "8 0" "8 248" "0 248" "0 0" "8 248" "8 0"; do
  set -- $cfg
  SFTAMD_BENCH_HOG_CUS=$1 SFTAMD_CU_BUDGET=$2 timeout -k 10 300 python bench.py > gpurun_out/r6_34_b.log 2>&1 || { tail -20 gpurun_out/r6_34_b.log; exit 1; }
  echo "held=$1 budget=$2 $(tail -1 gpurun_out/r6_34_b.log | cut -c60-140)" >> $out
done
cat $out
paste -d'\n' gpurun_out/r6_34_cu_b256.log gpurun_out/r6_34_cu_b248.log | grep -v amdgpu
