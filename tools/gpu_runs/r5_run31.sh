#!/bin/bash
# 4-wave kernel: read schedule A/B (B fragments first, no lgkmcnt(0) at the step start) on the step's backward shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_g4_layout.py > gpurun_out/r5_31_layout.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_31_layout.log | tail -60
exit $rc
