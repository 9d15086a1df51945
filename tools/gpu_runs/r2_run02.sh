#!/bin/bash
# Round 2: new GPU tests (bench self-launch), N=1 bench unchanged, cli.train with step phases + telemetry.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bench_gpu.py tests/test_ddp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_02_tests.log 2>&1 || { tail -40 gpurun_out/r2_02_tests.log; exit 1; }
tail -3 gpurun_out/r2_02_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_02_b1.log 2>&1 || { tail -20 gpurun_out/r2_02_b1.log; exit 1; }
grep metric gpurun_out/r2_02_b1.log
export OUTPUT_DIR=$GRAFT_REPO_ROOT/gpurun_out/r2_02_cli AIM_REPO=$GRAFT_REPO_ROOT/gpurun_out/r2_02_cli/aim BATCH_SIZE=8
timeout -k 10 400 python -m llm_fine_tune_distributed_amd.cli.train --model smollm3-3b --dataset synthetic --max-steps 12 --grad-accum 2 --freeze-policy full --no-gradient-checkpointing --log-step-phases --log-system-metrics-every 1 > gpurun_out/r2_02_cli.log 2>&1 || { tail -30 gpurun_out/r2_02_cli.log; exit 1; }
rm -rf gpurun_out/r2_02_cli/best_model gpurun_out/r2_02_cli/checkpoints/checkpoint-*
tail -5 gpurun_out/r2_02_cli.log
