#!/bin/bash
# round 6: single-pass cross-entropy (row in registers) vs the two-pass kernel: correctness, bandwidth, in-step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "ce" > gpurun_out/r6_17_tests.log 2>&1 || { tail -40 gpurun_out/r6_17_tests.log; exit 1; }
tail -2 gpurun_out/r6_17_tests.log
for r in 1 2; do
timeout -k 10 120 python -u tools/bench_ce.py > gpurun_out/r6_17_ce1_$r.log 2>&1 || { tail -20 gpurun_out/r6_17_ce1_$r.log; exit 1; }
echo "single $(tail -1 gpurun_out/r6_17_ce1_$r.log)"
SFTAMD_CE_TWO_PASS=1 timeout -k 10 120 python -u tools/bench_ce.py > gpurun_out/r6_17_ce2_$r.log 2>&1 || { tail -20 gpurun_out/r6_17_ce2_$r.log; exit 1; }
echo "two-pass $(tail -1 gpurun_out/r6_17_ce2_$r.log)"
done
