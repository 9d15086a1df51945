#!/bin/bash
# late-round evidence (after the 4-wave read-order change): kernel table of the headline step; PMC (MFMA busy, LDS
# conflicts) and HBM bytes of its kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof40s -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r5_40_ps.log 2>&1 || { tail -20 gpurun_out/r5_40_ps.log; exit 1; }
db=$(ls /tmp/prof40s/*/run_results.db /tmp/prof40s/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_40_step_prof.md > /dev/null
head -30 gpurun_out/r5_40_step_prof.md
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc40a -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r5_40_pmca.log 2>&1 || { tail -20 gpurun_out/r5_40_pmca.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc40b -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r5_40_pmcb.log 2>&1 || { tail -20 gpurun_out/r5_40_pmcb.log; exit 1; }
python tools/pmc_step.py /tmp/pmc40a /tmp/pmc40b --out gpurun_out/r5_40_step_pmc.md > /dev/null
head -30 gpurun_out/r5_40_step_pmc.md
