#!/bin/bash
# round 6: LDS bank conflicts / MFMA busy of the SwiGLU-fused down dgrad (cfg 7) vs its plain store and the 4-wave ring
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6_50.txt; : > $out
for case in "dgrad_down_swiglu 7" "dgrad_down 7" "dgrad_down 14"; do
  set -- $case
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc50_$1_$2 -o run -- python3 tools/pmc_gemm.py $1 $2 > gpurun_out/r6_50_$1_$2.log 2>&1 || { tail -20 gpurun_out/r6_50_$1_$2.log; exit 1; }
  echo "## $1 cfg $2" >> $out
  python tools/pmc_csv.py $(find /tmp/pmc50_$1_$2 -name "*counter_collection.csv") --match "dgrad,g4_kernel" >> $out
done
cat $out
