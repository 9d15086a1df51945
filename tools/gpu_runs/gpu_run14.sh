#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad" > gpurun_out/t16w.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t16w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/bw16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bw16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc16 -o pmc -- python tools/bench_wgrad.py --only gate_up --cfgs 1,3 --no-blas > gpurun_out/pmc16.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pmc16.log
exit 0
