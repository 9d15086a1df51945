#!/bin/bash
# small-output weight gradients (qkv, o): the 8-wave split rings vs the 4-wave kernel split over the tokens
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_wgrad.py --only qkv,o --cfgs 209,210,212,213,412,413,1213,1212 > gpurun_out/r4_41.log 2>&1 || { tail -20 gpurun_out/r4_41.log; exit 1; }
timeout -k 10 300 python -u tools/bench_wgrad.py --only qkv,o --cfgs 413,209,210,213,1213 --no-blas >> gpurun_out/r4_41.log 2>&1 || { tail -20 gpurun_out/r4_41.log; exit 1; }
grep shape gpurun_out/r4_41.log
