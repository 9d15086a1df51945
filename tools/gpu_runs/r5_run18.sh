#!/bin/bash
# per-op device time of 3 headline steps (torch.profiler inside bench.py: only the profiled steps, no init kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 5 --warmup 3 --profile-steps 3 --torch-profile gpurun_out/r5_18_ops.txt > gpurun_out/r5_18.log 2>&1 || { tail -20 gpurun_out/r5_18.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r5_18.log
head -60 gpurun_out/r5_18_ops.txt | cut -c1-260
