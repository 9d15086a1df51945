#!/bin/bash
# round 6: stream-K over the last partial round of the 4-wave weight-gradient GEMM (cfg 2014): correctness, then an
# interleaved A/B against each shape's current route
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py > gpurun_out/r6_07_tests.log 2>&1 || { tail -40 gpurun_out/r6_07_tests.log; exit 1; }
tail -2 gpurun_out/r6_07_tests.log
L=gpurun_out/r6_07_ab.log
: > $L
timeout -k 10 300 python -u tools/bench_ab.py wgrad gate_up 14,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad down 1214,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad qkv 1212,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad o 209,2014 >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad lm_head 1214,2014 --rounds 5 >> $L 2>&1 || { tail -30 $L; exit 1; }
grep kind $L
