#!/bin/bash
# round 6: in-step A/B of the forward projections on the row-contiguous HIP kernel (SFTAMD_FWD_GEMM=hip) vs the shipped
# TunableOp selections, with and without the overlapped AdamW (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in auto hip; do
for o in "" "--no-overlap"; do
  tag="${v}${o:+_noov}_$r"
  SFTAMD_FWD_GEMM=$v timeout -k 10 300 python -u bench.py $o > gpurun_out/r6_10_$tag.log 2>&1 || { tail -20 gpurun_out/r6_10_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r6_10_$tag.log | tr '\n' ' ')"
done; done; done
