#!/bin/bash
# Kernel profile of the recipe on the reference parquet (20 steps, 8 x GA 2 merged, eval at step 10): where the
# ~15 % per-token gap to bench.py at the same M goes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp OUTPUT_DIR=/tmp/sft_prof EPOCHS=1 BATCH_SIZE=8 AIM_REPO=/tmp/aim
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof67 -o run -- python -u -m llm_fine_tune_distributed_amd.cli.train \
  --dataset data/qa_dataset.parquet --freeze-policy full --grad-accum 2 --no-gradient-checkpointing --max-steps 20 \
  > gpurun_out/r2_67_p.log 2>&1 || { tail -30 gpurun_out/r2_67_p.log; exit 1; }
db=$(ls /tmp/prof67/*/run_results.db /tmp/prof67/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r2_67_prof.md > /dev/null
head -36 gpurun_out/r2_67_prof.md
