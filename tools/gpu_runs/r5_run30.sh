#!/bin/bash
# 4-wave kernel: the gate_up input gradient in its ROW / TR form vs the same product in the TR / TR form
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_g4_layout.py > gpurun_out/r5_30_layout.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_30_layout.log | tail -20
exit $rc
