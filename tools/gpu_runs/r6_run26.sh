#!/bin/bash
# round 6: flash attention's delta in the o_proj dgrad epilogue (dgrad_gemm_delta + the box hand-off): tests, step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_default_path_gpu.py > gpurun_out/r6_26_tests.log 2>&1 || { tail -40 gpurun_out/r6_26_tests.log; exit 1; }
tail -3 gpurun_out/r6_26_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/r6_26_bench$i.log 2>&1 || { tail -20 gpurun_out/r6_26_bench$i.log; exit 1; }
  tail -1 gpurun_out/r6_26_bench$i.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof26 -o run -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/r6_26_prof.log 2>&1 || { tail -20 gpurun_out/r6_26_prof.log; exit 1; }
find /tmp/prof26 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6_26_stats.csv \;
