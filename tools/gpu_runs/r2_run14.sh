#!/bin/bash
# Round 2: kernel trace of cli.train on synthetic Q&A (real chat-template token streams).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp BATCH_SIZE=8 OUTPUT_DIR=/tmp/cli_p AIM_REPO=/tmp/cli_p/aim
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_r2_14 -o run -- python -m llm_fine_tune_distributed_amd.cli.train --model smollm3-3b --dataset synthetic --max-steps 8 --grad-accum 2 --freeze-policy full --no-gradient-checkpointing --set eval_strategy=no --set save_strategy=no > gpurun_out/r2_14.log 2>&1 || { tail -20 gpurun_out/r2_14.log; exit 1; }
python tools/prof_summary.py $(find /tmp/prof_r2_14 -name "*.db" | head -1) --top 45 > gpurun_out/r2_14.md
echo ok
