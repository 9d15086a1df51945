#!/bin/bash
# RoPE backward fused into the attention backward (QKVRopeAttnFn / flash_bwd_rope): tests + bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash or rope" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_44_tests.log 2>&1 || { tail -40 gpurun_out/r2_44_tests.log; exit 1; }
tail -1 gpurun_out/r2_44_tests.log
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_44_tests2.log 2>&1 || { tail -40 gpurun_out/r2_44_tests2.log; exit 1; }
tail -1 gpurun_out/r2_44_tests2.log
for i in 1 2 3; do
  for p in 1 0; do
    SFTAMD_ROPE_ATTN=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_44_b$p.log 2>&1 || { tail -30 gpurun_out/r2_44_b$p.log; exit 1; }
    echo "ROPE_ATTN=$p $(tail -1 gpurun_out/r2_44_b$p.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["final_loss"])')"
  done
done
