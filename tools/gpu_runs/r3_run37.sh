#!/bin/bash
# attention: VALU-lean softmax in fwd3 / dK-dV v5 (packed fp32, one-compare masks, v_max3 tree): tests, A/B, PMC
# the attention microbench (stall / issue breakdown per kernel)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" \
  > gpurun_out/r3_37_test.log 2>&1 || { tail -40 gpurun_out/r3_37_test.log; exit 1; }
tail -1 gpurun_out/r3_37_test.log
B=16 ATTN_LEG=1 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r3_37_bench.log 2>&1 || { tail -30 gpurun_out/r3_37_bench.log; exit 1; }
B=16 RAGGED=1 ATTN_LEG=1 timeout -k 10 200 python -u tools/bench_attention.py >> gpurun_out/r3_37_bench.log 2>&1 || { tail -30 gpurun_out/r3_37_bench.log; exit 1; }
cat gpurun_out/r3_37_bench.log
cd /tmp
B=16 ATTN_QUICK=1 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace --output-format csv -d /tmp/apA -o run -- python $GRAFT_REPO_ROOT/tools/bench_attention.py > $GRAFT_REPO_ROOT/gpurun_out/r3_37_pa.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_37_pa.log; exit 1; }
B=16 ATTN_QUICK=1 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU \
  --kernel-trace --output-format csv -d /tmp/apB -o run -- python $GRAFT_REPO_ROOT/tools/bench_attention.py > $GRAFT_REPO_ROOT/gpurun_out/r3_37_pb.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_37_pb.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/pmc_step.py /tmp/apA --raw --top 12 --out gpurun_out/r3_37_pmcA.md > /dev/null
python tools/pmc_step.py /tmp/apB --raw --top 12 --out gpurun_out/r3_37_pmcB.md > /dev/null
cat gpurun_out/r3_37_pmcA.md gpurun_out/r3_37_pmcB.md
