#!/bin/bash
# round 6: the persistent forward 4-wave ring (gemm_tn cfg 70 / 71): correctness, interleaved A/B vs hipBLASLt and
# the row-contiguous pair-loop kernel (60 / 61)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_fwd_4wave or gemm_tn_rowc" > gpurun_out/r6_14_tests.log 2>&1 || { tail -40 gpurun_out/r6_14_tests.log; exit 1; }
tail -2 gpurun_out/r6_14_tests.log
L=gpurun_out/r6_14_ab.log
: > $L
timeout -k 10 400 python -u tools/bench_ab.py fwd gate_up,down,o,qkv blas,61,70,71 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py fwd lm_head blas,61,70,71 --rounds 5 >> $L 2>&1 || { tail -30 $L; exit 1; }
grep kind $L
