#!/bin/bash
# round 6: unsplit partial rounds vs token-split pieces for the o_proj + qkv pair alone and the lm_head wgrad
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug/partial_round_probe.py > gpurun_out/r6_74.log 2>&1 || { tail -20 gpurun_out/r6_74.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_74.log
