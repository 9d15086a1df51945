#!/bin/bash
# RCCL INFO log of a world-1 communicator through parallel/rccl_info.py (parser check on a real log)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe_rccl_info.py > gpurun_out/r5_36_rcclinfo.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_36_rcclinfo.log | tail -8
grep -h "Init COMPLETE\|nranks\|nRanks\|version\|Channel 00\|via " gpurun_out/rccl_info_probe/*.log | head -20
exit $rc
