#!/bin/bash
# round 6: stability of the final tree — 100 timed steps, and the overlapped update (the N > 1 default) on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*\|"loss_finite": [a-z]*' $1 | tr '\n' ' '; echo; }
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 > gpurun_out/r6_66_long.log 2>&1 || { tail -20 gpurun_out/r6_66_long.log; exit 1; }
echo "100 steps: $(v gpurun_out/r6_66_long.log)"
timeout -k 10 300 python -u bench.py --steps 20 --overlap on > gpurun_out/r6_66_overlap.log 2>&1 || { tail -20 gpurun_out/r6_66_overlap.log; exit 1; }
echo "overlap on: $(v gpurun_out/r6_66_overlap.log)"
timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_66_default.log 2>&1 || { tail -20 gpurun_out/r6_66_default.log; exit 1; }
echo "default: $(v gpurun_out/r6_66_default.log)"
