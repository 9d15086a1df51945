#!/bin/bash
# LoRA: dropout applied by bit selects, the scale folded into the fp32 results; timings + tests + bench + profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 env PYTHONPATH=. python -u tools/bench_lora_kernels.py > gpurun_out/r4_50_k.log 2>&1 && cat gpurun_out/r4_50_k.log &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_trainer_gpu.py -k "lora" > gpurun_out/r4_50_tests.log 2>&1 || { tail -30 gpurun_out/r4_50_tests.log; exit 1; }
tail -2 gpurun_out/r4_50_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_50_lora.log 2>&1 || { tail -20 gpurun_out/r4_50_lora.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_50_lora.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof50 -o run -- python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/r4_50_p.log 2>&1 || { tail -20 gpurun_out/r4_50_p.log; exit 1; }
db=$(ls /tmp/prof50/*/run_results.db /tmp/prof50/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r4_50_lora_prof.md > /dev/null
head -45 gpurun_out/r4_50_lora_prof.md
