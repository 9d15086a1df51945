#!/bin/bash
# round 6: attention A/B, previous build (_C_ab_old.so: mask as selects, scalar bf16 packing) vs this tree's _C.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_23_attn.log; : > $out
for i in 1 2 3; do
  for v in old new; do
    lib=llm_fine_tune_distributed_amd/_C.so; [ $v = old ] && lib=llm_fine_tune_distributed_amd/_C_ab_old.so
    echo "== $v $i" >> $out
    SFTAMD_LIB=$lib B=16 CFGS=ds ROUNDS=5 timeout -k 10 120 python -u tools/bench_attention.py >> $out 2>&1 || { tail -20 $out; exit 1; }
    SFTAMD_LIB=$lib B=16 RAGGED=1 CFGS=ds ROUNDS=5 timeout -k 10 120 python -u tools/bench_attention.py >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
cat $out
