#!/bin/bash
# 4-wave backward GEMMs: read schedule with the B fragments first and no lgkmcnt(0) at the step start
# (SFTAMD_G4_FB=1, temporary) vs the current schedule, in the step (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SFTAMD_G4_FB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py > gpurun_out/r5_32_tests.log 2>&1 || { tail -30 gpurun_out/r5_32_tests.log; exit 1; }
tail -1 gpurun_out/r5_32_tests.log
for v in 1 0 1 0; do
  SFTAMD_G4_FB=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_32_fb$v.log 2>&1 || { tail -20 gpurun_out/r5_32_fb$v.log; exit 1; }
  echo "fb $v $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_32_fb$v.log | tr '\n' ' ')"
done
