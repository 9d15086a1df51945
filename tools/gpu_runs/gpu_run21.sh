#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof21_lora -o run -- python bench.py --steps 4 --warmup 2 --freeze-policy lora --no-overlap > gpurun_out/p21_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p21_lora.log; [ $rc -eq 0 ] || exit $rc
B=16 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc21 -o pmc -- python tools/bench_attention.py > gpurun_out/pmc21.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pmc21.log
