#!/bin/bash
# round 6: AdamW grid-stride window vs contiguous range per block (one SmolLM3 region, 1.54e9 parameters)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_adamw_layout.py > gpurun_out/r6_38.log 2>&1 || { tail -20 gpurun_out/r6_38.log; exit 1; }
cat gpurun_out/r6_38.log
