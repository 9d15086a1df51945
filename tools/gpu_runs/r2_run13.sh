#!/bin/bash
# Round 2: where does cli.train lose vs bench.py? logging cadence / phases / eval off.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export BATCH_SIZE=8
c() {
  tag=$1; shift
  OUTPUT_DIR=/tmp/cli_$tag AIM_REPO=/tmp/cli_$tag/aim timeout -k 10 400 python -m llm_fine_tune_distributed_amd.cli.train --model smollm3-3b --dataset synthetic --max-steps 24 --grad-accum 2 --freeze-policy full --no-gradient-checkpointing "$@" > gpurun_out/r2_13_$tag.log 2>&1 || { tail -30 gpurun_out/r2_13_$tag.log; exit 1; }
  echo "$tag $(grep -o 'train_pure_samples_per_second=[0-9.]*' gpurun_out/r2_13_$tag.log | tail -1) $(grep -o 'train_runtime=[0-9.]*' gpurun_out/r2_13_$tag.log | tail -1)"
}
c default
c nolog_noeval --set logging_steps=1000 --set eval_strategy=no --set save_strategy=no
c noeval --set eval_strategy=no --set save_strategy=no
c bf16m_nolog --set logging_steps=1000 --set eval_strategy=no --set save_strategy=no --set optim_state_dtype=bf16
