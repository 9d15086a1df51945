#!/bin/bash
# 4-wave GEMM (cfg 12): timing-only ablations (1201 no DMA, 1202 no fragment reads, 1204 no barrier, 1203 neither
# DMA nor reads) and PMC passes vs hipBLASLt on gate_up.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 12,1201,1202,1203,1204,11 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,gu8k:22016:8192 > gpurun_out/r3_02_abl.log 2>&1 || { tail -30 gpurun_out/r3_02_abl.log; exit 1; }
cat gpurun_out/r3_02_abl.log
for c in 12 blas 11; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/pmc_$c -o run -- python tools/pmc_tn.py $c > gpurun_out/r3_02_pmc_$c.log 2>&1 || { tail -5 gpurun_out/r3_02_pmc_$c.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d /tmp/pmc2_$c -o run -- python tools/pmc_tn.py $c >> gpurun_out/r3_02_pmc_$c.log 2>&1 || { tail -5 gpurun_out/r3_02_pmc_$c.log; exit 1; }
  for d in pmc pmc2; do f=$(find /tmp/${d}_$c -name "*counter_collection.csv" | head -1); cp $f gpurun_out/r3_02_${d}_$c.csv; done
  python tools/pmc_csv.py gpurun_out/r3_02_pmc_$c.csv gpurun_out/r3_02_pmc2_$c.csv --match tn4_kernel,Cijk,tn3_kernel
done
