#!/bin/bash
# round 6: attention backward with the mask as a real branch + one-instruction bf16 pair packing: tests, kernel time, step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_gemm_4w_gpu.py > gpurun_out/r6_22_tests.log 2>&1 || { tail -30 gpurun_out/r6_22_tests.log; exit 1; }
tail -3 gpurun_out/r6_22_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof22 -o run -- python3 tools/pmc_attn.py > gpurun_out/r6_22b.log 2>&1 || { tail -20 gpurun_out/r6_22b.log; exit 1; }
find /tmp/prof22 -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 > gpurun_out/r6_22_stats.csv
head -8 gpurun_out/r6_22_stats.csv
timeout -k 10 300 python bench.py > gpurun_out/r6_22_bench1.log 2>&1 || { tail -20 gpurun_out/r6_22_bench1.log; exit 1; }
tail -1 gpurun_out/r6_22_bench1.log
timeout -k 10 300 python bench.py > gpurun_out/r6_22_bench2.log 2>&1 || { tail -20 gpurun_out/r6_22_bench2.log; exit 1; }
tail -1 gpurun_out/r6_22_bench2.log
