#!/bin/bash
# round 6: full GPU suite after the CU-budget / cu_hog changes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_35_tests.log 2>&1 || { tail -40 gpurun_out/r6_35_tests.log; exit 1; }
tail -1 gpurun_out/r6_35_tests.log
