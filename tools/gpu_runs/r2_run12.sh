#!/bin/bash
# Round 2: cli.train on synthetic Q&A (ragged lengths) with auto pad-to-64 vs exact padding; secondary bench configs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export BATCH_SIZE=8
for pm in auto exact; do
  extra=""
  if [ $pm = exact ]; then extra="--set pad_to_multiple_of=1"; fi
  OUTPUT_DIR=/tmp/cli_$pm AIM_REPO=/tmp/cli_$pm/aim timeout -k 10 400 python -m llm_fine_tune_distributed_amd.cli.train --model smollm3-3b --dataset synthetic --max-steps 14 --grad-accum 2 --freeze-policy full --no-gradient-checkpointing --log-step-phases $extra > gpurun_out/r2_12_cli_$pm.log 2>&1 || { tail -30 gpurun_out/r2_12_cli_$pm.log; exit 1; }
  cp /tmp/cli_$pm/training_history.json gpurun_out/r2_12_hist_$pm.json
  grep "train_runtime" gpurun_out/r2_12_cli_$pm.log | tail -1
done
: > gpurun_out/r2_12_bench.jsonl
run() {
  tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/r2_12_$tag.log 2>&1 || { tail -20 gpurun_out/r2_12_$tag.log; exit 1; }
  grep metric gpurun_out/r2_12_$tag.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['tag']='$tag'; print(json.dumps(r))" >> gpurun_out/r2_12_bench.jsonl
  tail -1 gpurun_out/r2_12_bench.jsonl | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['tag'], r['value'], r['ms_per_step'], r['peak_mem_gb'])"
}
run lora --freeze-policy lora --steps 10 --warmup 3
run last_n_layers --freeze-policy last_n_layers --steps 10 --warmup 3
run packing --packing --steps 10 --warmup 3
run llama3_8b --model llama3-8b --steps 5 --warmup 2
