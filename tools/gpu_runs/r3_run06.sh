#!/bin/bash
# default-path whole-model test at SmolLM3 widths (dispatch trace), IPC all-reduce hardening, 4-wave GEMM tests,
# then the fused SwiGLU / RoPE epilogues of the 4-wave kernel vs hipBLASLt + separate kernels and cfg 11
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_env_guard.py tests/test_default_path_gpu.py \
  tests/test_ipc_allreduce_gpu.py > gpurun_out/r3_06_test.log 2>&1 || { tail -60 gpurun_out/r3_06_test.log; exit 1; }
grep -E "PASS|FAIL|uncached" gpurun_out/r3_06_test.log | tail -12
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn" \
  > gpurun_out/r3_06_k.log 2>&1 || { tail -40 gpurun_out/r3_06_k.log; exit 1; }
tail -2 gpurun_out/r3_06_k.log
for m in 8192 10240; do
timeout -k 10 300 python -u tools/bench_gemm_tn.py --fused-cfgs 11,12,50 --m $m --iters 30 > gpurun_out/r3_06_$m.log 2>&1 || { tail -30 gpurun_out/r3_06_$m.log; exit 1; }
cat gpurun_out/r3_06_$m.log
done
