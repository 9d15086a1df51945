#!/bin/bash
# LoRA step under torch.profiler: which ops launch the small fill / copy kernels
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 2 --warmup 3 --profile-steps 2 --freeze-policy lora --torch-profile gpurun_out/r4_39_torchprof.txt > gpurun_out/r4_39.log 2>&1 || { tail -20 gpurun_out/r4_39.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_39.log
