#!/bin/bash
# qkv weight gradient on the 4-wave kernel split over the tokens (cfg 1212): default-path / model tests + bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_default_path_gpu.py tests/test_model_gpu.py tests/test_gemm_4w_gpu.py tests/test_trainer_gpu.py > gpurun_out/r4_42_tests.log 2>&1 || { tail -30 gpurun_out/r4_42_tests.log; exit 1; }
tail -1 gpurun_out/r4_42_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_42_bench.log 2>&1 || { tail -20 gpurun_out/r4_42_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_42_bench.log
