#!/bin/bash
# LoRA wide forward GEMM shapes (K + 128 columns): which forward-layout config
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python -u tools/bench_gemm_tn.py --plain-only --cfgs 164,11,12,2 --shapes "qkv_nope:3072:2176,o:2048:2176,gate_up:22016:2176,down:2048:11136" > gpurun_out/r4_53_$i.log 2>&1 || { tail -20 gpurun_out/r4_53_$i.log; exit 1; }
grep "^|" gpurun_out/r4_53_$i.log
done
