#!/bin/bash
# Plain projections (o_proj, NoPE qkv) on the BK64 HIP GEMM: model-level numerics, then interleaved bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t46.log 2>&1 || { tail -30 gpurun_out/t46.log; exit 1; }
tail -2 gpurun_out/t46.log
: > gpurun_out/b46.log
for r in 1 2; do
  for v in 1 0; do
    echo "TN_PLAIN=$v" >> gpurun_out/b46.log
    SFTAMD_TN_PLAIN=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric >> gpurun_out/b46.log || exit 1
  done
done
python - <<'PY'
import json
cur = None
for l in open("gpurun_out/b46.log"):
    if l.startswith("TN_PLAIN"): cur = l.strip()
    else: print(cur, json.loads(l)["value"])
PY
