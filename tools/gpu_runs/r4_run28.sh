#!/bin/bash
# LoRA forward widening: what the A-operand loads cost (timing-only variant without them, SFTAMD_LORA_NOA)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_28_a.log 2>&1 && cat gpurun_out/r4_28_a.log &&
SFTAMD_LORA_NOA=1 timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_28_b.log 2>&1 && cat gpurun_out/r4_28_b.log
