#!/bin/bash
# the driver's smoke() on the final tree
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_54_smoke.log 2>&1 || { tail -20 gpurun_out/r4_54_smoke.log; exit 1; }
tail -3 gpurun_out/r4_54_smoke.log
