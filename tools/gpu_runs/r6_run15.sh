#!/bin/bash
# round 6: forward gate_up PMC: hipBLASLt vs tn6 (61) vs the forward ring (70)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in blas 61 70; do
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc15_$v -o run -- python3 tools/bench_ab.py fwd gate_up $v --rounds 1 --iters 3 > gpurun_out/r6_15_$v.log 2>&1 || { tail -20 gpurun_out/r6_15_$v.log; exit 1; }
echo "== $v"
python tools/pmc_csv.py $(find /tmp/pmc15_$v -name "*counter_collection.csv") --match "Cijk,tn6_kernel,g4f_kernel" | tee -a gpurun_out/r6_15_pmc.txt
done
