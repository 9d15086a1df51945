#!/bin/bash
# round 6: cost of the delta epilogue on the o_proj dgrad (interleaved A/B), attention backward with / without delta
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_ab.py dgrad o,qkv 14,delta --rounds 9 > gpurun_out/r6_28_ab.log 2>&1 || { tail -20 gpurun_out/r6_28_ab.log; exit 1; }
cat gpurun_out/r6_28_ab.log
B=16 CFGS=ds,dsd ROUNDS=7 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r6_28_attn.log 2>&1 || { tail -20 gpurun_out/r6_28_attn.log; exit 1; }
cat gpurun_out/r6_28_attn.log
