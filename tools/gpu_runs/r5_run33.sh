#!/bin/bash
# forward projections on the 4-wave kernel's ROW / ROW form (gemm_tn cfg 70 / 71) vs cfg 60 and hipBLASLt (tuned)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_fwd_g4.py > gpurun_out/r5_33_fwd.log 2>&1
rc=$?
grep -v "amdgpu.ids" gpurun_out/r5_33_fwd.log | tail -20
exit $rc
