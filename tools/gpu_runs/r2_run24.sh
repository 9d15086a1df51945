#!/bin/bash
# Ping-pong TN GEMM: K sweep (fixed per-tile cost vs per-K cost) and PMC passes (clock, MFMA busy, waits).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_gemm_tn.py --cfgs 5,9,11 --plain-only --shapes gu1k:22016:1024,gu2k:22016:2048,gu4k:22016:4096,gu8k:22016:8192,sq8k:8192:8192 2>&1 | tee gpurun_out/r2_24_ksweep.md
for c in 11 blas; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d /tmp/pmc_$c -o run -- python tools/pmc_tn.py $c > gpurun_out/r2_24_pmc_$c.log 2>&1 || { tail -5 gpurun_out/r2_24_pmc_$c.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d /tmp/pmc2_$c -o run -- python tools/pmc_tn.py $c >> gpurun_out/r2_24_pmc_$c.log 2>&1 || { tail -5 gpurun_out/r2_24_pmc_$c.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d /tmp/pmc3_$c -o run -- python tools/pmc_tn.py $c >> gpurun_out/r2_24_pmc_$c.log 2>&1 || { tail -5 gpurun_out/r2_24_pmc_$c.log; exit 1; }
  for d in pmc pmc2 pmc3; do f=$(find /tmp/${d}_$c -name "*counter_collection.csv" | head -1); cp $f gpurun_out/r2_24_${d}_$c.csv; done
done
ls gpurun_out | grep r2_24
