#!/bin/bash
# per-kernel PMC table of the end-of-round-3 default step (after the attention and epilogue work): two passes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --kernel-trace --output-format csv -d /tmp/pmc50A -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_50_a.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_50_a.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc50B -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_50_b.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_50_b.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/pmc_step.py /tmp/pmc50A /tmp/pmc50B --out gpurun_out/r3_50_pmc.md > /dev/null
head -40 gpurun_out/r3_50_pmc.md
