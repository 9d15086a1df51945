#!/bin/bash
# Optimizer side stream restricted to n CUs (hipExtStreamCreateWithCUMask): same-box interleaved bench sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
b() {  # tag env...
  tag=$1; shift
  v=$(env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*') || exit 1
  echo "$tag $v"
}
for r in 1 2; do
  b all SFTAMD_ADAMW_CUS=0
  b cu16 SFTAMD_ADAMW_CUS=16
  b cu32 SFTAMD_ADAMW_CUS=32
  b cu32s8 SFTAMD_ADAMW_CUS=32 SFTAMD_ADAMW_CU_STRIDE=8
  b cu64 SFTAMD_ADAMW_CUS=64
  b cu64s4 SFTAMD_ADAMW_CUS=64 SFTAMD_ADAMW_CU_STRIDE=4
  b cu128 SFTAMD_ADAMW_CUS=128
done
