#!/bin/bash
# qkv / o weight-gradient configs at the bench's and the recipe's token counts (routing check for cfg 1213 / 213)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in 8192 10240; do
  timeout -k 10 200 python -u tools/bench_wgrad.py --tokens $T --cfgs 210,209,1213,213,13 --only qkv,o --no-blas > gpurun_out/r3_49_$T.log 2>&1 || { tail -30 gpurun_out/r3_49_$T.log; exit 1; }
  grep -v "^\[" gpurun_out/r3_49_$T.log | tail -8
done
