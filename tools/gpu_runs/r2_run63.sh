#!/bin/bash
# The reference recipe end to end on its own dataset (data/qa_dataset.parquet, 2845 Q&A rows -> 2560 / 285 split):
# cli.train, full-parameter SFT, 8 x GA 2, one epoch, eval every 10 steps, final save. Random-init SmolLM3-3B and
# the offline tokenizer (no hub access on the box).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export OUTPUT_DIR=/tmp/sft_run EPOCHS=1 BATCH_SIZE=8 AIM_REPO=/tmp/aim
timeout -k 10 900 python -u -m llm_fine_tune_distributed_amd.cli.train --dataset data/qa_dataset.parquet \
  --freeze-policy full --grad-accum 2 --no-gradient-checkpointing --log-step-phases > gpurun_out/r2_63_train.log 2>&1 || { tail -40 gpurun_out/r2_63_train.log; exit 1; }
cp /tmp/sft_run/training_summary.json gpurun_out/r2_63_training_summary.json
cp /tmp/sft_run/training_history.json gpurun_out/r2_63_training_history.json
tail -5 gpurun_out/r2_63_train.log
cat gpurun_out/r2_63_training_summary.json
