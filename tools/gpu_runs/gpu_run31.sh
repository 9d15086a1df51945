#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/s31.log
for G in 1 4 8 16 32; do
  SFTAMD_TN_GROUP=$G timeout -k 10 120 python tools/sweep_tn.py >> gpurun_out/s31.log 2>&1 || exit $?
done
