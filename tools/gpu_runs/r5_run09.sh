#!/bin/bash
# round 5: dxa kernel with 512-column chunks; the plain row-contiguous gate_up GEMM per kernel in the step (no overlap)
# vs hipBLASLt; the reference recipe A/B + kernel table; LoRA with the new defaults
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -k "dxa or lora or rowc" > gpurun_out/r5_09_tests.log 2>&1 || { tail -40 gpurun_out/r5_09_tests.log; exit 1; }
tail -1 gpurun_out/r5_09_tests.log
timeout -k 10 200 python -u tools/bench_lora_dxa.py > gpurun_out/r5_09_dxa.log 2>&1 || { tail -20 gpurun_out/r5_09_dxa.log; exit 1; }
cat gpurun_out/r5_09_dxa.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r5_09_lora.log 2>&1 || { tail -20 gpurun_out/r5_09_lora.log; exit 1; }
echo "lora $(grep -o '"value": [0-9.]*' gpurun_out/r5_09_lora.log)"
SFTAMD_TN_CFG=60 SFTAMD_FWD_HIP_N=22016 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof09 -o run -- python bench.py --steps 6 --warmup 2 --no-overlap > gpurun_out/r5_09_p.log 2>&1 || { tail -20 gpurun_out/r5_09_p.log; exit 1; }
db=$(ls /tmp/prof09/*/run_results.db /tmp/prof09/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_09_step_prof_gu60.md > /dev/null
head -20 gpurun_out/r5_09_step_prof_gu60.md
bash tools/gpu_runs/r5_run07.sh
