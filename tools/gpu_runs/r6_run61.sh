#!/bin/bash
# round 6: a layer's o_proj + qkv weight gradients carried into the previous layer's MLP launch (four-problem grid):
# GPU tests, then the step interleaved against SFTAMD_WGRAD_CARRY=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py -m gpu > gpurun_out/r6_61_tests.log 2>&1 || { tail -40 gpurun_out/r6_61_tests.log; exit 1; }
tail -1 gpurun_out/r6_61_tests.log
timeout -k 10 200 python -u tools/bench_pair.py --pair attn --splits 3 > gpurun_out/r6_61_pair.log 2>&1 || { tail -20 gpurun_out/r6_61_pair.log; exit 1; }
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for r in 1 0; do
SFTAMD_WGRAD_CARRY=$r timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_61_b${r}_$i.log 2>&1 || { tail -20 gpurun_out/r6_61_b${r}_$i.log; exit 1; }
echo "carry=$r $i: $(v gpurun_out/r6_61_b${r}_$i.log)"
done
done
