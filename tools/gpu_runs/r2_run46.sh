#!/bin/bash
# Secondary configs on the current kernels: LoRA, the reference freeze policy, Llama-3-8B, packing, fp32 moments.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 "$@" > gpurun_out/r2_46_$tag.log 2>&1 || { tail -30 gpurun_out/r2_46_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r2_46_$tag.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["tokens_per_sec"], r.get("mfu"), r["peak_mem_gb"])')"
}
run default
run lora --freeze-policy lora
run refpolicy --freeze-policy last_n_layers
run packing --packing
run fp32m --optim-state fp32
run ga2split --micro-batch 8 --ga 2 --ga-merge-max-tokens 0
run llama8b --model llama3-8b
