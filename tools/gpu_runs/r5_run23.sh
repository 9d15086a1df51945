#!/bin/bash
# end-of-round evidence: rocprofv3 kernel tables of the headline step and the LoRA step; PMC (MFMA busy, LDS
# conflicts) and HBM bytes of the headline step's kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof23s -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r5_23_ps.log 2>&1 || { tail -20 gpurun_out/r5_23_ps.log; exit 1; }
db=$(ls /tmp/prof23s/*/run_results.db /tmp/prof23s/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r5_23_step_prof.md > /dev/null
head -30 gpurun_out/r5_23_step_prof.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof23l -o run -- python bench.py --freeze-policy lora --steps 6 --warmup 2 > gpurun_out/r5_23_pl.log 2>&1 || { tail -20 gpurun_out/r5_23_pl.log; exit 1; }
db=$(ls /tmp/prof23l/*/run_results.db /tmp/prof23l/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 50 --out gpurun_out/r5_23_lora_prof.md > /dev/null
head -40 gpurun_out/r5_23_lora_prof.md
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc23a -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r5_23_pmca.log 2>&1 || { tail -20 gpurun_out/r5_23_pmca.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc23b -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r5_23_pmcb.log 2>&1 || { tail -20 gpurun_out/r5_23_pmcb.log; exit 1; }
python tools/pmc_step.py /tmp/pmc23a /tmp/pmc23b --out gpurun_out/r5_23_step_pmc.md > /dev/null
head -30 gpurun_out/r5_23_step_pmc.md
