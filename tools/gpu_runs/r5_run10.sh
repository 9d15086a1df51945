#!/bin/bash
# round 5: full GPU suite + smoke on the new defaults (shape-aware forward routing, LoRA wide cfg 61, dxa kernel)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r5_10_tests.log 2>&1 || { tail -60 gpurun_out/r5_10_tests.log; exit 1; }
tail -2 gpurun_out/r5_10_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_10_smoke.log 2>&1 || { tail -20 gpurun_out/r5_10_smoke.log; exit 1; }
tail -1 gpurun_out/r5_10_smoke.log
