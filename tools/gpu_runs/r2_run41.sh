#!/bin/bash
# Coarser optimizer-update waits in the forward (SFTAMD_UPDATE_WAIT_STRIDE): bench A/B (final_loss must match).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  for p in 4 1; do
    SFTAMD_UPDATE_WAIT_STRIDE=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_41_b$p.log 2>&1 || { tail -30 gpurun_out/r2_41_b$p.log; exit 1; }
    echo "STRIDE=$p $(tail -1 gpurun_out/r2_41_b$p.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["final_loss"])')"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_41_t.log 2>&1 || { tail -30 gpurun_out/r2_41_t.log; exit 1; }
tail -1 gpurun_out/r2_41_t.log
