#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_ddp_gpu.py -x -q -m gpu > gpurun_out/t7.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t7.log; ok $rc
timeout -k 10 500 python bench.py --steps 4 --warmup 2 --model llama3-8b > gpurun_out/b7_llama.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b7_llama.log; ok $rc
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --freeze-policy lora > gpurun_out/b7_lora.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b7_lora.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-master-weights > gpurun_out/b7_nomaster.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b7_nomaster.log; ok $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "L rc=$?" >> gpurun_out/counters.txt
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc7a -o run --output-format csv -- python3 tools/bench_attention.py > gpurun_out/pmc7a.log 2>&1; echo "rc=$?" >> gpurun_out/pmc7a.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d gpurun_out/pmc7b -o run --output-format csv -- python3 tools/bench_attention.py > gpurun_out/pmc7b.log 2>&1; echo "rc=$?" >> gpurun_out/pmc7b.log
