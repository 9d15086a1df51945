#!/bin/bash
# round 6: qkv / o weight gradients: the pair-loop split (1212) and 8-wave split (209) vs the interleaved ring split
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r6_08_ab.log
: > $L
timeout -k 10 300 python -u tools/bench_ab.py wgrad qkv 1212,1214,214,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad o 209,214,414,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
grep kind $L
