#!/bin/bash
# SwiGLU dgrad epilogue with a 8-deep gate/up register ring: tests, microbench, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py -k "swiglu or dgrad or default" \
  > gpurun_out/r3_44_test.log 2>&1 || { tail -40 gpurun_out/r3_44_test.log; exit 1; }
tail -1 gpurun_out/r3_44_test.log
DGRAD_CFGS=7 timeout -k 10 200 python -u tools/bench_dgrad.py > gpurun_out/r3_44_dg.log 2>&1 || { tail -30 gpurun_out/r3_44_dg.log; exit 1; }
grep -v "^\[" gpurun_out/r3_44_dg.log | tail -12
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_44_bench.log 2>&1 || { tail -20 gpurun_out/r3_44_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_44_bench.log | cut -c1-200
