#!/bin/bash
# LoRA forward widening: row-contiguous LDS-staged kernel (SFTAMD_LORA_FWD2) vs the fragment-layout one
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SFTAMD_LORA_FWD2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora" > gpurun_out/r4_29_t.log 2>&1 || { tail -30 gpurun_out/r4_29_t.log; exit 1; }
tail -1 gpurun_out/r4_29_t.log
timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_29_a.log 2>&1 && grep fwd gpurun_out/r4_29_a.log &&
SFTAMD_LORA_FWD2=1 timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_29_b.log 2>&1 && grep fwd gpurun_out/r4_29_b.log
