#!/bin/bash
# RCCL communicator with 2 ranks on one MI355X (probe)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe_rccl2.py > gpurun_out/r5_34_rccl2.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_34_rccl2.log | tail -30
exit $rc
