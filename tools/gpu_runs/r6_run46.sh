#!/bin/bash
# round 6: the NoPE layers' o_proj + qkv pair too: tests (+ model) + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_model_gpu.py tests/test_default_path_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py > gpurun_out/r6_46_tests.log 2>&1 || { tail -40 gpurun_out/r6_46_tests.log; exit 1; }
tail -2 gpurun_out/r6_46_tests.log
out=gpurun_out/r6_46.log; : > $out
for v in 1 0 1 0 1 0; do
  SFTAMD_WGRAD_PAIR=$v timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r6_46_b.log 2>&1 || { tail -20 gpurun_out/r6_46_b.log; exit 1; }
  echo "pair=$v $(grep -o '"value": [0-9.]*' gpurun_out/r6_46_b.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r6_46_b.log)" >> $out
done
cat $out
