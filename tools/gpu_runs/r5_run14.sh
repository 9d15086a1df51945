#!/bin/bash
# round 5: AdamW launch shapes (UNR 4) and SR cost
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_adamw.py > gpurun_out/r5_14_adamw.log 2>&1 || { tail -20 gpurun_out/r5_14_adamw.log; exit 1; }
grep moments gpurun_out/r5_14_adamw.log
bash tools/gpu_runs/r5_run15.sh
