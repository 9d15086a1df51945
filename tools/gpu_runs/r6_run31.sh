#!/bin/bash
# round 6: attention backward PMC after the mask branch + packed conversions
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d /tmp/pmc31 -o run -- python3 tools/pmc_attn.py > gpurun_out/r6_31.log 2>&1 || { tail -20 gpurun_out/r6_31.log; exit 1; }
python tools/pmc_csv.py $(find /tmp/pmc31 -name "*counter_collection.csv") --match "fwd32,dkdv32,dq32,delta" | tee gpurun_out/r6_31_pmc.txt
