#!/bin/bash
# LoRA streaming kernels (final): PMC passes + per-kernel times
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pa52 -o run -- python tools/pmc_lora.py > gpurun_out/r4_52_pa.log 2>&1 || { tail -5 gpurun_out/r4_52_pa.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d /tmp/pb52 -o run -- python tools/pmc_lora.py > gpurun_out/r4_52_pb.log 2>&1 || { tail -5 gpurun_out/r4_52_pb.log; exit 1; }
python tools/pmc_csv.py $(ls /tmp/pa52/*/run_counter_collection.csv /tmp/pa52/run_counter_collection.csv /tmp/pb52/*/run_counter_collection.csv /tmp/pb52/run_counter_collection.csv 2>/dev/null) --match "fwd_kernel<1, true>,fwd_kernel<3, false>,bwd_dx,swiglu_fwd,tsum_kernel<1, 4>,tsum_kernel<2, 4>" > gpurun_out/r4_52_pmc.txt
cat gpurun_out/r4_52_pmc.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/pc52 -o run -- python tools/pmc_lora.py > gpurun_out/r4_52_pc.log 2>&1 || { tail -5 gpurun_out/r4_52_pc.log; exit 1; }
f=$(ls /tmp/pc52/*/run_kernel_stats.csv /tmp/pc52/run_kernel_stats.csv 2>/dev/null | head -1); cut -d, -f1-4 $f
