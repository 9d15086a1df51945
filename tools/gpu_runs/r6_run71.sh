#!/bin/bash
# round 6: final check of the committed tree — the whole GPU suite as the driver runs it, smoke, the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_71_tests.log 2>&1 || { tail -40 gpurun_out/r6_71_tests.log; exit 1; }
tail -1 gpurun_out/r6_71_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_71_smoke.log 2>&1 || { tail -20 gpurun_out/r6_71_smoke.log; exit 1; }
tail -1 gpurun_out/r6_71_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6_71_bench.log 2>&1 || { tail -20 gpurun_out/r6_71_bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"loss_finite": [a-z]*' gpurun_out/r6_71_bench.log | tr '\n' ' '; echo
