#!/bin/bash
# Hardware counters of the training step, one rocprofv3 --pmc pass each (MFMA / LDS, then HBM reads).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmcA -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r2_51_a.log 2>&1 || { tail -20 gpurun_out/r2_51_a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmcB -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r2_51_b.log 2>&1 || { tail -20 gpurun_out/r2_51_b.log; exit 1; }
python tools/pmc_step.py /tmp/pmcA /tmp/pmcB --top 30 --out gpurun_out/r2_51_pmc.md
ls /tmp/pmcA | head; find /tmp/pmcA -name "*.csv" | head -5
