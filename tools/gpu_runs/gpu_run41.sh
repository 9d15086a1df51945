#!/bin/bash
# End-to-end product check on one MI355X: reference-compatible training.py (env contract, reference
# SFTConfig: last-2-layers policy, GA 4, grad checkpointing, eval every 10 steps, best model) on the
# synthetic Q&A set for 20 optimizer steps, then the inference CLI on the saved best_model.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e
export EPOCHS=1 BATCH_SIZE=8 OUTPUT_DIR=$GRAFT_REPO_ROOT/gpurun_out/e2e AIM_REPO=/tmp/aim_e2e
timeout -k 10 600 python -u training.py --dataset synthetic --max-steps 20 > gpurun_out/e2e_train.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/e2e_train.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/e2e/checkpoints
ls -la gpurun_out/e2e gpurun_out/e2e/best_model >> gpurun_out/e2e_train.log 2>&1
timeout -k 10 300 python -u ask_tuned_model.py "How do I tie a bowline?" --model gpurun_out/e2e/best_model --max-new-tokens 48 --seed 1 > gpurun_out/e2e_ask.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/e2e_ask.log
rm -f gpurun_out/e2e/best_model/*.safetensors
