#!/bin/bash
# in-step kernel times of the fused gate_up + SwiGLU (cfg 50) vs hipBLASLt + the SwiGLU kernel, and the recipe profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SFTAMD_GATE_UP=50 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof29 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r3_29_p.log 2>&1 || { tail -20 gpurun_out/r3_29_p.log; exit 1; }
db=$(ls /tmp/prof29/*/run_results.db /tmp/prof29/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 30 --out gpurun_out/r3_29_prof.md > /dev/null
head -24 gpurun_out/r3_29_prof.md
bash tools/gpu_runs/r3_run28.sh
