#!/bin/bash
# round 6: plain + SwiGLU input gradients re-routed to the conflict-free 8-wave ring (cfg 5); GPU tests of the
# dispatch, then the step interleaved against SFTAMD_DGRAD_RING8=0 (old routing for plain dgrads, cfg 5 for SwiGLU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_default_path_gpu.py tests/test_kernels_gpu.py tests/test_gemm_4w_gpu.py tests/test_model_gpu.py -m gpu > gpurun_out/r6_54_tests.log 2>&1 || { tail -40 gpurun_out/r6_54_tests.log; exit 1; }
tail -1 gpurun_out/r6_54_tests.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for r in 1 0; do
SFTAMD_DGRAD_RING8=$r timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_54_b${r}_$i.log 2>&1 || { tail -20 gpurun_out/r6_54_b${r}_$i.log; exit 1; }
echo "ring8=$r $i: $(v gpurun_out/r6_54_b${r}_$i.log)"
done
done
