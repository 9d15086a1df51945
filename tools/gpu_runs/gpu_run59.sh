#!/bin/bash
# Tune the Llama-3-8B training GEMM shapes into the shipped selections, then re-measure that config.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model llama3-8b --steps 3 --warmup 2 2>&1 | grep metric > gpurun_out/llama59_before.log || exit 1
PYTORCH_TUNABLEOP_VERBOSE=3 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 timeout -k 10 1000 python bench.py --model llama3-8b --steps 1 --warmup 1 --tunableop tune > gpurun_out/tune59.log 2>&1 || { tail -5 gpurun_out/tune59.log; exit 1; }
cp tuning/tunableop_results_mi355x.csv gpurun_out/tuned59.csv
timeout -k 10 300 python bench.py --model llama3-8b --steps 3 --warmup 2 2>&1 | grep metric > gpurun_out/llama59_after.log || exit 1
python -c "
import json
for f in ('before','after'): print(f, json.loads(open(f'gpurun_out/llama59_{f}.log').read())['value'])"
wc -l gpurun_out/tuned59.csv
