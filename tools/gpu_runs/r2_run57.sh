#!/bin/bash
# Weight-gradient partial last round on a side stream (SFTAMD_WGRAD_STREAM=tail): tests + bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_57_tests.log 2>&1 || { tail -40 gpurun_out/r2_57_tests.log; exit 1; }
tail -1 gpurun_out/r2_57_tests.log
for i in 1 2 3; do
  for p in tail 0; do
    SFTAMD_WGRAD_STREAM=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_57_b$p.log 2>&1 || { tail -30 gpurun_out/r2_57_b$p.log; exit 1; }
    echo "WGRAD_STREAM=$p $(tail -1 gpurun_out/r2_57_b$p.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["final_loss"])')"
  done
done
