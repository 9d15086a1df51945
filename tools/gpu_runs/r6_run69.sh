#!/bin/bash
# round 6: is a residual add free inside the hipBLASLt forward (addmm with beta = 1) at the o / down shapes?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/debug/addmm_probe.py > gpurun_out/r6_69.log 2>&1 || { tail -20 gpurun_out/r6_69.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_69.log
