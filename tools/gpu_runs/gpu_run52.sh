#!/bin/bash
# Gradient norm summed per bucket during backward (side stream) vs the post-backward pass: GPU tests + bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t52.log 2>&1 || { tail -30 gpurun_out/t52.log; exit 1; }
tail -2 gpurun_out/t52.log
: > gpurun_out/b52.log
for r in 1 2; do
  for v in 1 0; do
    echo "NORM_IN_BWD=$v" >> gpurun_out/b52.log
    SFTAMD_NORM_IN_BWD=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric >> gpurun_out/b52.log || exit 1
  done
done
python - <<'PY'
import json
cur = None
for l in open("gpurun_out/b52.log"):
    if l.startswith("NORM"): cur = l.strip()
    else: print(cur, json.loads(l)["value"])
PY
