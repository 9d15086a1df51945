#!/bin/bash
# forward GEMMs with the weight's row pitch padded, each (shape, pitch) TunableOp-tuned in-process
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 50; do echo "[tune] still running $(date +%T)"; done ) &
HB=$!
timeout -k 10 1000 python -u tools/bench_wpitch.py > gpurun_out/r5_29_wpitch.log 2>&1
rc=$?
kill $HB
grep -v "amdgpu.ids" gpurun_out/r5_29_wpitch.log | tail -20
exit $rc
