#!/bin/bash
# attention schedule fixes (vm_drain before the loop, lse multiply pinned after the prefetch, dq4 scratch gone,
# permlane reductions): correctness, then same-process A/B vs the round-2 schedule at 16 x 512 and the recipe's
# ragged 16 x ~621, then a kernel profile of the default path
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" \
  > gpurun_out/r3_35_test.log 2>&1 || { tail -40 gpurun_out/r3_35_test.log; exit 1; }
tail -2 gpurun_out/r3_35_test.log
B=16 ATTN_LEG=1 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r3_35_bench.log 2>&1 || { tail -30 gpurun_out/r3_35_bench.log; exit 1; }
cat gpurun_out/r3_35_bench.log
B=16 RAGGED=1 ATTN_LEG=1 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r3_35_bench_rag.log 2>&1 || { tail -30 gpurun_out/r3_35_bench_rag.log; exit 1; }
cat gpurun_out/r3_35_bench_rag.log
