#!/bin/bash
# 4-wave backward GEMMs (csrc/gemm_4w.hip): correctness vs fp32, then wgrad / dgrad microbench vs the 8-wave rings
# and hipBLASLt at the SmolLM3 shapes (T = M = 8192)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py \
  > gpurun_out/r3_14_test.log 2>&1 || { tail -40 gpurun_out/r3_14_test.log; exit 1; }
tail -2 gpurun_out/r3_14_test.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 10,9,209,210,12,13,213,1213,1313 > gpurun_out/r3_14_wgrad.log 2>&1 || { tail -30 gpurun_out/r3_14_wgrad.log; exit 1; }
grep '^{' gpurun_out/r3_14_wgrad.log
DGRAD_CFGS=7,12,13 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r3_14_dgrad.log 2>&1 || { tail -30 gpurun_out/r3_14_dgrad.log; exit 1; }
grep '^{' gpurun_out/r3_14_dgrad.log
DGRAD_SHAPES=lm_head DGRAD_CFGS=12,13 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r3_14_dgrad2.log 2>&1 || { tail -30 gpurun_out/r3_14_dgrad2.log; exit 1; }
grep '^{' gpurun_out/r3_14_dgrad2.log
