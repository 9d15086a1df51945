#!/bin/bash
# Round 3, first GPU call: the 4-wave 128x128 forward GEMM (cfg 12) — correctness, then timing vs hipBLASLt and
# the 8-wave ping-pong (cfg 11) at the SmolLM3 projection shapes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave or gemm_tn_plain" \
  > gpurun_out/r3_01_test.log 2>&1 || { tail -40 gpurun_out/r3_01_test.log; exit 1; }
tail -3 gpurun_out/r3_01_test.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 11,12 --plain-only --iters 30 > gpurun_out/r3_01_bench.log 2>&1 || { tail -30 gpurun_out/r3_01_bench.log; exit 1; }
cat gpurun_out/r3_01_bench.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 11,12 --plain-only --iters 30 --m 10240 > gpurun_out/r3_01_bench2.log 2>&1 || { tail -30 gpurun_out/r3_01_bench2.log; exit 1; }
cat gpurun_out/r3_01_bench2.log
