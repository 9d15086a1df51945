#!/bin/bash
# attention: three-stage LDS-DMA forward ring: tests, A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" \
  > gpurun_out/r3_46_test.log 2>&1 || { tail -40 gpurun_out/r3_46_test.log; exit 1; }
tail -1 gpurun_out/r3_46_test.log
B=16 ROUNDS=5 ATTN_LEG=1 timeout -k 10 250 python -u tools/bench_attention.py > gpurun_out/r3_46_bench.log 2>&1 || { tail -30 gpurun_out/r3_46_bench.log; exit 1; }
B=16 ROUNDS=5 RAGGED=1 ATTN_LEG=1 timeout -k 10 250 python -u tools/bench_attention.py >> gpurun_out/r3_46_bench.log 2>&1 || { tail -30 gpurun_out/r3_46_bench.log; exit 1; }
cat gpurun_out/r3_46_bench.log
