#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b33.log
for mode in 0 rope swiglu 1; do
  for ov in "" "--no-overlap"; do
    echo "TN=$mode $ov" >> gpurun_out/b33.log
    SFTAMD_TN=$mode timeout -k 10 300 python bench.py --steps 10 --warmup 3 --optim-state bf16 $ov 2>&1 | grep metric >> gpurun_out/b33.log || exit 1
  done
done
