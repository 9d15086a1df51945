#!/bin/bash
# per-kernel PMC table of the round-3 default step (MFMA busy, clock, LDS bank conflicts, HBM reads): two passes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --kernel-trace --output-format csv -d /tmp/pmcA -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_34_a.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_34_a.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmcB -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r3_34_b.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_34_b.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/pmc_step.py /tmp/pmcA /tmp/pmcB --out gpurun_out/r3_34_pmc.md > /dev/null
head -40 gpurun_out/r3_34_pmc.md
