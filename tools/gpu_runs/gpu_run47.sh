#!/bin/bash
# Attention backward: dq kernel concurrently with dK/dV on a side stream. Tests, microbench, bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/t47.log 2>&1 || { tail -30 gpurun_out/t47.log; exit 1; }
tail -2 gpurun_out/t47.log
B=16 ATTN_QUICK=1 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/a47.log 2>&1 || { tail -20 gpurun_out/a47.log; exit 1; }
grep impl gpurun_out/a47.log
: > gpurun_out/b47.log
for r in 1 2; do
  for v in 1 0; do
    echo "CONC=$v" >> gpurun_out/b47.log
    SFTAMD_ATTN_CONC=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric >> gpurun_out/b47.log || exit 1
  done
done
python - <<'PY'
import json
cur = None
for l in open("gpurun_out/b47.log"):
    if l.startswith("CONC"): cur = l.strip()
    else: print(cur, json.loads(l)["value"])
PY
