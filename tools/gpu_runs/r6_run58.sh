#!/bin/bash
# round 6: SwiGLU-fused down dgrad on 256 x 128 tiles (cfg 2: 73 KB LDS, 133 VGPRs -> two workgroups per CU, whose
# epilogues can overlap each other's main loops) vs 256 x 256 (cfg 5, 7)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DGRAD_CFGS=5,2,7 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r6_58.log 2>&1 || { tail -20 gpurun_out/r6_58.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_58.log
