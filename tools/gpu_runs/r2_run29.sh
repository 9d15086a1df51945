#!/bin/bash
# Fused gradient norm, take 2 (no extra ring-kernel argument): tests, kernel profile of the step, A/B vs base.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "norm_slots or sumsq_chunks or wgrad_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_29_tests.log 2>&1 || { tail -40 gpurun_out/r2_29_tests.log; exit 1; }
tail -1 gpurun_out/r2_29_tests.log
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -k "fused_grad_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_29_tests2.log 2>&1 || { tail -40 gpurun_out/r2_29_tests2.log; exit 1; }
tail -1 gpurun_out/r2_29_tests2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof29 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r2_29_p.log 2>&1 || { tail -20 gpurun_out/r2_29_p.log; exit 1; }
db=$(ls /tmp/prof29/*/run_results.db /tmp/prof29/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 30 --out gpurun_out/r2_29_prof.md > /dev/null
R=3 bash tools/gpu_runs/r2_ab.sh
