#!/bin/bash
# LoRA on the hand-written path: GPU tests, bench (HIP forward vs hipBLASLt forward), kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py -k "lora" > gpurun_out/r4_09_tests.log 2>&1 || { tail -30 gpurun_out/r4_09_tests.log; exit 1; }
tail -2 gpurun_out/r4_09_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_09_lora.log 2>&1 || { tail -20 gpurun_out/r4_09_lora.log; exit 1; }
grep '"metric"' gpurun_out/r4_09_lora.log
SFTAMD_LORA_FWD=blas timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_09_lora_blas.log 2>&1 || { tail -20 gpurun_out/r4_09_lora_blas.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_09_lora_blas.log | sed 's/^/lora blas fwd /'
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof09 -o run -- python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/r4_09_p.log 2>&1 || { tail -20 gpurun_out/r4_09_p.log; exit 1; }
db=$(ls /tmp/prof09/*/run_results.db /tmp/prof09/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r4_09_lora_prof.md > /dev/null
head -60 gpurun_out/r4_09_lora_prof.md
