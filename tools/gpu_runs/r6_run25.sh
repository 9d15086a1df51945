#!/bin/bash
# round 6: attention A/B, HEAD build (_C_ab_old.so) vs this tree (uniform dS^T store flag)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_25_attn.log; : > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or flash" > gpurun_out/r6_25_tests.log 2>&1 || { tail -30 gpurun_out/r6_25_tests.log; exit 1; }
tail -2 gpurun_out/r6_25_tests.log
for i in 1 2 3; do
  for v in old new; do
    lib=llm_fine_tune_distributed_amd/_C.so; [ $v = old ] && lib=llm_fine_tune_distributed_amd/_C_ab_old.so
    echo "== $v $i" >> $out
    SFTAMD_LIB=$lib B=16 CFGS=ds ROUNDS=5 timeout -k 10 120 python -u tools/bench_attention.py >> $out 2>&1 || { tail -20 $out; exit 1; }
    SFTAMD_LIB=$lib B=16 RAGGED=1 CFGS=ds ROUNDS=5 timeout -k 10 120 python -u tools/bench_attention.py >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
cat $out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof25 -o run -- python3 tools/pmc_attn.py > gpurun_out/r6_25b.log 2>&1 || { tail -20 gpurun_out/r6_25b.log; exit 1; }
find /tmp/prof25 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6_25_stats.csv \;
cut -d, -f1-8 gpurun_out/r6_25_stats.csv | head -8
