#!/bin/bash
# final check of the committed tree: full GPU suite + smoke + one headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5_41_tests.log 2>&1 || { tail -40 gpurun_out/r5_41_tests.log; exit 1; }
tail -2 gpurun_out/r5_41_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_41_smoke.log 2>&1 || { tail -20 gpurun_out/r5_41_smoke.log; exit 1; }
tail -1 gpurun_out/r5_41_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5_41_bench.log 2>&1 || { tail -20 gpurun_out/r5_41_bench.log; exit 1; }
grep '"metric"' gpurun_out/r5_41_bench.log
