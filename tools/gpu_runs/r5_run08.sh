#!/bin/bash
# round 5: plain-store row-contiguous forward GEMM (cfg 60: the output stays cacheable for the consumer) in the step;
# LoRA dxa kernel tests + microbench; LoRA wide GEMM cfg 164 / 61 / 60; default-path + LoRA-overlap tests; Llama-3-8B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_trainer_gpu.py tests/test_default_path_gpu.py -m gpu -k "dxa or lora_overlap or default_path or overlap_matches or swiglu_bwd" > gpurun_out/r5_08_tests.log 2>&1 || { tail -40 gpurun_out/r5_08_tests.log; exit 1; }
tail -1 gpurun_out/r5_08_tests.log
timeout -k 10 200 python -u tools/bench_lora_dxa.py > gpurun_out/r5_08_dxa.log 2>&1 || { tail -20 gpurun_out/r5_08_dxa.log; exit 1; }
cat gpurun_out/r5_08_dxa.log
run() {
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r5_08_$n.log 2>&1 || { tail -20 gpurun_out/r5_08_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r5_08_$n.log)"
}
for r in 1 2; do
  run base$r X=1 --
  run gu60_$r SFTAMD_TN_CFG=60 SFTAMD_FWD_HIP_N=22016 --
  run fused60_$r SFTAMD_TN=1 SFTAMD_TN_CFG=60 --
done
run lora164 X=1 -- --freeze-policy lora
run lora61 SFTAMD_LORA_FWD_CFG=61 -- --freeze-policy lora
run lora60 SFTAMD_LORA_FWD_CFG=60 -- --freeze-policy lora
run llama X=1 -- --model llama3-8b --steps 10 --warmup 3
grep '"metric"' gpurun_out/r5_08_llama.log | cut -c1-300
