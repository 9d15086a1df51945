#!/bin/bash
# round 6: interleaved A/B of the 4-wave ring issue variants (14 both interleaved, 15 reads only, 16 DMA only; 12xx =
# hybrid split of the last partial round) on the step's backward GEMMs; lm_head wgrad vs the 8-wave cfg 10
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r6_05_ab.log
: > $L
timeout -k 10 300 python -u tools/bench_ab.py wgrad gate_up,down 14,1214,15,1215,16,1216 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad lm_head 10,14,1214,1215,1216 --rounds 5 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py dgrad gate_up,down,lm_head 14,15,16,blas --rounds 5 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py dgrad o,qkv 12,14,15,16 >> $L 2>&1 || { tail -30 $L; exit 1; }
cat $L
