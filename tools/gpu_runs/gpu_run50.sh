#!/bin/bash
# AdamW launch shape: unrolled loads (UNR 1 vs 2) x block cap, isolated bandwidth, then end-to-end A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "adamw" -x -q --timeout 120 --timeout-method thread > gpurun_out/t50.log 2>&1 || { tail -30 gpurun_out/t50.log; exit 1; }
tail -2 gpurun_out/t50.log
timeout -k 10 300 python tools/bench_adamw.py > gpurun_out/adam50.log 2>&1 || { tail -20 gpurun_out/adam50.log; exit 1; }
grep UNR gpurun_out/adam50.log
: > gpurun_out/b50.log
for r in 1 2; do
  for v in "1 2048" "2 2048" "2 4096"; do
    set -- $v
    echo "UNR=$1 BLOCKS=$2" >> gpurun_out/b50.log
    SFTAMD_ADAM_UNR=$1 SFTAMD_ADAM_BLOCKS=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric >> gpurun_out/b50.log || exit 1
  done
done
python - <<'PY'
import json
cur = None
for l in open("gpurun_out/b50.log"):
    if l.startswith("UNR"): cur = l.strip()
    else: print(cur, json.loads(l)["value"])
PY
