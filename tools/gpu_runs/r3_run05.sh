#!/bin/bash
# 4-wave GEMM (cfg 12 = VAR 4) with the fused SwiGLU / RoPE epilogues vs hipBLASLt + the separate kernels and cfg 11
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave or gemm_tn_swiglu or gemm_tn_rope" \
  > gpurun_out/r3_05_test.log 2>&1 || { tail -40 gpurun_out/r3_05_test.log; exit 1; }
tail -2 gpurun_out/r3_05_test.log
for m in 8192 10240; do
timeout -k 10 300 python -u tools/bench_gemm_tn.py --fused-cfgs 11,12 --m $m --iters 30 > gpurun_out/r3_05_$m.log 2>&1 || { tail -30 gpurun_out/r3_05_$m.log; exit 1; }
cat gpurun_out/r3_05_$m.log
done
