#!/bin/bash
# small weight-gradient configs (o_proj, qkv) sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_small_wgrad.py > gpurun_out/r5_39_wgrad.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_39_wgrad.log | tail -30
exit $rc
