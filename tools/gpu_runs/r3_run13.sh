#!/bin/bash
# re-entry checkpoint: default bench (20 steps) with a kernel profile, then r3_run12 (attention v6 tests + timing,
# chunked LM head test, persistent GEMM A/B)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_13_bench.log 2>&1 || { tail -30 gpurun_out/r3_13_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_13_bench.log
bash tools/gpu_runs/r3_run12.sh
