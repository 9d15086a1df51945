#!/bin/bash
# Ping-pong forward GEMM in the fused epilogues: tests, then same-box interleaved bench variants vs the base commit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_27_tests.log 2>&1 || { tail -40 gpurun_out/r2_27_tests.log; exit 1; }
tail -1 gpurun_out/r2_27_tests.log
b() {  # tag dir env...
  tag=$1; d=$2; shift 2
  v=$(cd $d && env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*') || exit 1
  echo "$tag $v"
}
for r in 1 2; do
  b new $GRAFT_REPO_ROOT SFTAMD_TN=rope
  b new_tn1 $GRAFT_REPO_ROOT SFTAMD_TN=1
  b new_tn1_plain $GRAFT_REPO_ROOT SFTAMD_TN=1 SFTAMD_TN_PLAIN=1
  b base $GRAFT_REPO_ROOT/_ab_base SFTAMD_TN=rope
done
