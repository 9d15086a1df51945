#!/bin/bash
# round 6: natural-order reads in the BK = 32 ring too (cfg 2 tail, cfg 5): tests, PMC, A/B vs the cfg-7-only build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py -k "dgrad or default_path" > gpurun_out/r6_52_tests.log 2>&1 || { tail -40 gpurun_out/r6_52_tests.log; exit 1; }
tail -2 gpurun_out/r6_52_tests.log
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc52 -o run -- python3 tools/pmc_gemm.py dgrad_down_swiglu 7 > gpurun_out/r6_52_pmc.log 2>&1 || { tail -20 gpurun_out/r6_52_pmc.log; exit 1; }
python tools/pmc_csv.py $(find /tmp/pmc52 -name "*counter_collection.csv") --match "dgrad" | tee gpurun_out/r6_52_pmc.txt
out=gpurun_out/r6_52_ab.log; : > $out
for i in 1 2 3; do
  for v in old new; do
    lib=llm_fine_tune_distributed_amd/_C.so; [ $v = old ] && lib=llm_fine_tune_distributed_amd/_C_ab_old.so
    SFTAMD_LIB=$lib DGRAD_CFGS=7,5 timeout -k 10 200 python -u tools/bench_dgrad.py --rounds 3 > gpurun_out/r6_52_b.log 2>&1 || { tail -20 gpurun_out/r6_52_b.log; exit 1; }
    echo "== $v $i $(grep -h 'swiglu\|down' gpurun_out/r6_52_b.log | tr '\n' ' ')" >> $out
  done
done
cat $out
