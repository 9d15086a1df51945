#!/bin/bash
# Refresh the secondary BASELINE configs on the current kernels: LoRA, reference partial-freeze policy,
# Llama-3-8B full SFT (1 GPU; the 8-GPU run is the driver's).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b44.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --freeze-policy lora 2>&1 | grep metric >> gpurun_out/b44.log || exit 1
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --freeze-policy last_n_layers 2>&1 | grep metric >> gpurun_out/b44.log || exit 1
timeout -k 10 500 python bench.py --steps 4 --warmup 2 --model llama3-8b 2>&1 | grep metric >> gpurun_out/b44.log || exit 1
