#!/bin/bash
# round 6: the four-problem weight-gradient grid's leftover split count (the _multi_split cost model's check)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_pair.py --pair layer --splits 1,2,3,4,5,6,8 --rounds 9 > gpurun_out/r6_72.log 2>&1 || { tail -20 gpurun_out/r6_72.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_72.log
