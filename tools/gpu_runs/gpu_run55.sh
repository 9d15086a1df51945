#!/bin/bash
# Full GPU suite + smoke + headline bench (x2) on the current tree.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t55.log 2>&1 || { tail -30 gpurun_out/t55.log; exit 1; }
tail -2 gpurun_out/t55.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s55.log 2>&1 || { tail -20 gpurun_out/s55.log; exit 1; }
tail -1 gpurun_out/s55.log
for r in 1 2; do
  timeout -k 10 300 python bench.py 2>&1 | grep metric >> gpurun_out/b55.log || exit 1
done
python -c "
import json
for l in open('gpurun_out/b55.log'): print(json.loads(l)['value'], json.loads(l)['ms_per_step'])"
