#!/bin/bash
# Step-start critical path: token count via the pinned batch path + cached padded-batch metadata (always on
# here), and the AdamW block cap under the overlapped forward (SFTAMD_ADAM_BLOCKS A/B, interleaved).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t49.log 2>&1 || { tail -30 gpurun_out/t49.log; exit 1; }
tail -2 gpurun_out/t49.log
: > gpurun_out/b49.log
for r in 1 2; do
  for v in 2048 512 256 128; do
    echo "ADAM_BLOCKS=$v" >> gpurun_out/b49.log
    SFTAMD_ADAM_BLOCKS=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric >> gpurun_out/b49.log || exit 1
  done
done
python - <<'PY'
import json
cur = None
for l in open("gpurun_out/b49.log"):
    if l.startswith("ADAM"): cur = l.strip()
    else: print(cur, json.loads(l)["value"])
PY
