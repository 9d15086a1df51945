#!/bin/bash
# gate_up input with a padded row pitch (the norm writes it into a wider buffer; gate_up then runs on the
# row-contiguous kernel, its wgrad reads x through the pitch): in-step A/B vs the default (hipBLASLt, tuned)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py > gpurun_out/r5_28_tests.log 2>&1 || { tail -30 gpurun_out/r5_28_tests.log; exit 1; }
tail -1 gpurun_out/r5_28_tests.log
for v in 64 0 128 64 0 128; do
  SFTAMD_GU_PAD=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_28_pad$v.log 2>&1 || { tail -20 gpurun_out/r5_28_pad$v.log; exit 1; }
  echo "pad $v $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_28_pad$v.log | tr '\n' ' ')"
done
