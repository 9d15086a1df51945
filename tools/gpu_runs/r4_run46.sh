#!/bin/bash
# LoRA streaming kernels: what the regenerated dropout mask costs the dA reduction
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_46_k.log 2>&1 && cat gpurun_out/r4_46_k.log
