#!/bin/bash
# round 5: row-contiguous forward GEMM (cfg 60 / 61) correctness + microbench vs hipBLASLt / cfg 164
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "rowc or 4wave" > gpurun_out/r5_01_tests.log 2>&1 || { tail -40 gpurun_out/r5_01_tests.log; exit 1; }
tail -2 gpurun_out/r5_01_tests.log
timeout -k 10 200 python -u tools/bench_gemm_tn.py --cfgs 164,60,61 --plain-only > gpurun_out/r5_01_plain.log 2>&1 || { tail -20 gpurun_out/r5_01_plain.log; exit 1; }
cat gpurun_out/r5_01_plain.log
timeout -k 10 200 python -u tools/bench_gemm_tn.py --fused-cfgs 164,60,61 > gpurun_out/r5_01_fused.log 2>&1 || { tail -20 gpurun_out/r5_01_fused.log; exit 1; }
cat gpurun_out/r5_01_fused.log
timeout -k 10 200 python -u tools/bench_gemm_tn.py --m 10240 --fused-cfgs 164,60,61 > gpurun_out/r5_01_fused10k.log 2>&1 || { tail -20 gpurun_out/r5_01_fused10k.log; exit 1; }
cat gpurun_out/r5_01_fused10k.log
