#!/bin/bash
# round 6: headline kernel table of the timed steps and a per-kernel PMC pass after the four-problem weight-gradient grids
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof64 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_64_ps.log 2>&1 || { tail -20 gpurun_out/r6_64_ps.log; exit 1; }
db=$(ls /tmp/prof64/*/run_results.db /tmp/prof64/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --window adamw_kernel 4 --title "headline step, timed steps only" --out gpurun_out/r6_64_steps.md > /dev/null
head -30 gpurun_out/r6_64_steps.md
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc64 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r6_64_pmc.log 2>&1 || { tail -20 gpurun_out/r6_64_pmc.log; exit 1; }
python tools/pmc_step.py /tmp/pmc64 --out gpurun_out/r6_64_pmc.md > /dev/null && head -40 gpurun_out/r6_64_pmc.md
