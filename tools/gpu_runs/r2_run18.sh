#!/bin/bash
# Round 2: PMC counters of the attention kernels.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pa -o run -- python tools/pmc_attn.py > gpurun_out/r2_18.log 2>&1 || { tail -5 gpurun_out/r2_18.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/pb -o run -- python tools/pmc_attn.py >> gpurun_out/r2_18.log 2>&1 || { tail -5 gpurun_out/r2_18.log; exit 1; }
cp $(find /tmp/pa -name "*counter_collection.csv") gpurun_out/r2_18_a.csv
cp $(find /tmp/pb -name "*counter_collection.csv") gpurun_out/r2_18_b.csv
echo ok
