#!/bin/bash
# Round 2: PMC counters of the ring GEMM mainloops (one pass per counter group, each under its own time limit).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in "wgrad_down 9" "wgrad_gateup 10" "dgrad_down 1"; do
  set -- $k
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pmc_$1 -o run -- python tools/pmc_gemm.py $1 $2 > gpurun_out/r2_15_$1.log 2>&1 || { tail -5 gpurun_out/r2_15_$1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/pmc2_$1 -o run -- python tools/pmc_gemm.py $1 $2 >> gpurun_out/r2_15_$1.log 2>&1 || { tail -5 gpurun_out/r2_15_$1.log; exit 1; }
  find /tmp/pmc_$1 /tmp/pmc2_$1 -name "*counter_collection.csv" -exec cp {} gpurun_out/ \; -exec sh -c 'mv gpurun_out/$(basename $1) gpurun_out/r2_15_'$1'_$(basename $(dirname $1))_$(basename $1)' _ {} \;
done
ls gpurun_out | grep r2_15
