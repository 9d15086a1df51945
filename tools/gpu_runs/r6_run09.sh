#!/bin/bash
# round 6: after pruning the unrouted GEMM variants and re-routing (qkv / o wgrad on the 4-wave split, lm_head hybrid,
# every plain dgrad on cfg 14): full GPU suite, then the headline bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_default_path_gpu.py > gpurun_out/r6_09_dp.log 2>&1 || { tail -40 gpurun_out/r6_09_dp.log; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_09_tests.log 2>&1 || { tail -40 gpurun_out/r6_09_tests.log; exit 1; }
tail -2 gpurun_out/r6_09_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py > gpurun_out/r6_09_bench$i.log 2>&1 || { tail -20 gpurun_out/r6_09_bench$i.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r6_09_bench$i.log | tr '\n' ' '; echo
done
