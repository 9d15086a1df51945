#!/bin/bash
# round 6: 4-wave wgrad time vs tile count (is a partial last round a full round's time?)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug/round_scaling.py > gpurun_out/r6_43.log 2>&1 || { tail -20 gpurun_out/r6_43.log; exit 1; }
cat gpurun_out/r6_43.log
