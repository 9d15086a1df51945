#!/bin/bash
# Round-4 baseline: default bench, forward GEMM microbench (hipBLASLt vs persistent 4-wave cfg 50) at M = 8192 / 10240
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_01_bench.log 2>&1 || { tail -20 gpurun_out/r4_01_bench.log; exit 1; }
grep '"metric"' gpurun_out/r4_01_bench.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 12,50,60,61 --plain-only > gpurun_out/r4_01_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_01_gemm8k.log; exit 1; }
cat gpurun_out/r4_01_gemm8k.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 10240 --cfgs 12,50 --plain-only > gpurun_out/r4_01_gemm10k.log 2>&1 || { tail -20 gpurun_out/r4_01_gemm10k.log; exit 1; }
cat gpurun_out/r4_01_gemm10k.log
