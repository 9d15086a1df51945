#!/bin/bash
# round 6: AdamW flat update bandwidth: current kernel vs nontemporal streams, block caps, and the byte-mix ceiling
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r6_11_adamw.log
: > $L
for r in 1 2; do
for v in 0 1 2 3 4 5; do
  echo "variant $v" >> $L
  SFTAMD_ADAMW_VARIANT=$v timeout -k 10 120 python -u tools/bench_adamw.py >> $L 2>&1 || { tail -20 $L; exit 1; }
done; done
cat $L
