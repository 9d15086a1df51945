#!/bin/bash
# round 6: re-check the failed default-path test (cfg 14 names) + the LoRA in-place widening ranks; lm_head wgrad
# routing (8-wave cfg 10 vs the 4-wave ring 14 / hybrid 1214, both orders); SwiGLU dgrad cfg 7 vs g4 cfg 14; torch
# profiler attribution of the step's ATen glue
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_default_path_gpu.py tests/test_model_gpu.py -k "default_path or lora_norm" > gpurun_out/r6_04_tests.log 2>&1 || { tail -40 gpurun_out/r6_04_tests.log; exit 1; }
tail -2 gpurun_out/r6_04_tests.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 10,14,1214 --only lm_head --no-blas > gpurun_out/r6_04_wg1.log 2>&1 || { tail -30 gpurun_out/r6_04_wg1.log; exit 1; }
grep shape gpurun_out/r6_04_wg1.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 1214,14,10 --only lm_head --no-blas > gpurun_out/r6_04_wg2.log 2>&1 || { tail -30 gpurun_out/r6_04_wg2.log; exit 1; }
grep shape gpurun_out/r6_04_wg2.log
DGRAD_CFGS=7,14 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r6_04_dgrad.log 2>&1 || { tail -30 gpurun_out/r6_04_dgrad.log; exit 1; }
tail -6 gpurun_out/r6_04_dgrad.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --profile-steps 3 --torch-profile gpurun_out/r6_04_torchprof.txt > gpurun_out/r6_04_bench.log 2>&1 || { tail -30 gpurun_out/r6_04_bench.log; exit 1; }
grep '"metric"' gpurun_out/r6_04_bench.log | cut -c1-300
