#!/bin/bash
# attention A/B (fwd32 vs fwd3, dkdv32 vs dkdv5) + per-kernel times + PMC passes of the default path
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or flash or attn" > gpurun_out/r4_14_attn.log 2>&1 || { tail -40 gpurun_out/r4_14_attn.log; exit 1; }
tail -2 gpurun_out/r4_14_attn.log
B=16 timeout -k 10 300 python -u tools/bench_attention.py > gpurun_out/r4_14_bench.log 2>&1 || { tail -20 gpurun_out/r4_14_bench.log; exit 1; }
cat gpurun_out/r4_14_bench.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/p14a -o run -- python tools/pmc_attn.py > gpurun_out/r4_14_pa.log 2>&1 || { tail -5 gpurun_out/r4_14_pa.log; exit 1; }
SFTAMD_ATTN_DKDV5=1 SFTAMD_ATTN_FWD16=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/p14b -o run -- python tools/pmc_attn.py > gpurun_out/r4_14_pb.log 2>&1 || { tail -5 gpurun_out/r4_14_pb.log; exit 1; }
for d in p14a p14b; do f=$(ls /tmp/$d/*/run_kernel_stats.csv /tmp/$d/run_kernel_stats.csv 2>/dev/null | head -1); echo "== $d"; cut -d, -f1-4 $f | grep -i "attn\|Name" ; cp $f gpurun_out/r4_14_${d}_stats.csv; done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pc -o run -- python tools/pmc_attn.py > gpurun_out/r4_14_pc.log 2>&1 || { tail -5 gpurun_out/r4_14_pc.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/pd -o run -- python tools/pmc_attn.py >> gpurun_out/r4_14_pc.log 2>&1 || { tail -5 gpurun_out/r4_14_pc.log; exit 1; }
python tools/pmc_csv.py $(ls /tmp/pc/*/run_counter_collection.csv /tmp/pc/run_counter_collection.csv /tmp/pd/*/run_counter_collection.csv /tmp/pd/run_counter_collection.csv 2>/dev/null) --match fwd32,dkdv32,dq32,delta > gpurun_out/r4_14_pmc.txt
cat gpurun_out/r4_14_pmc.txt
