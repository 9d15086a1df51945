#!/bin/bash
# Cross-entropy row stream with 4 loads in flight per thread: numerics, isolated A/B, bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "cross_entropy or lm_head or loss" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_59_tests.log 2>&1 || { tail -40 gpurun_out/r2_59_tests.log; exit 1; }
tail -1 gpurun_out/r2_59_tests.log
for u in 1 4 1 4; do
  echo "CE_UNROLL=$u $(SFTAMD_CE_UNROLL=$u timeout -k 10 120 python tools/bench_ce.py)" || exit 1
done
for i in 1 2; do
  for u in 4 1; do
    SFTAMD_CE_UNROLL=$u timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_59_b$u.log 2>&1 || { tail -30 gpurun_out/r2_59_b$u.log; exit 1; }
    echo "bench CE_UNROLL=$u $(tail -1 gpurun_out/r2_59_b$u.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["final_loss"])')"
  done
done
