#!/bin/bash
# qkv + RoPE forward: cfg 11 (+ tail split, the default) vs the persistent 164 and 12, and vs hipBLASLt + kernel
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python -u tools/bench_gemm_tn.py --fused-cfgs 11,164,12,2 > gpurun_out/r4_44_$i.log 2>&1 || { tail -20 gpurun_out/r4_44_$i.log; exit 1; }
grep "RoPE" gpurun_out/r4_44_$i.log
done
