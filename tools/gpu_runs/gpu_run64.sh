#!/bin/bash
# Refresh of the secondary README configs on the current kernels (one box, sequential).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b64.log
run() {
  tag=$1; shift
  v=$(timeout -k 10 300 python bench.py "$@" 2>&1 | grep metric) || { echo "FAIL $tag"; exit 1; }
  echo "$v" | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['note']='gpu_run64 $tag'; print(json.dumps(r))" >> gpurun_out/b64.log
  echo "$tag $(echo "$v" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['tokens_per_sec'], r['peak_mem_gb'])")"
}
run default
run bf16_moments --optim-state bf16
run master_weights --master-weights
run ref_split_mb8_ga2 --micro-batch 8 --ga 2
run lora --freeze-policy lora
run last_n_layers --freeze-policy last_n_layers
run packing --packing
