#!/bin/bash
# round 6 experiment: the 8-wave BK-32 dgrad ring with sched_group_barrier interleave (cfg 6) vs without (cfg 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_ab.py dgrad down,gate_up,qkv 5,6 --rounds 7 > gpurun_out/r6_79_ab.log 2>&1 || { tail -20 gpurun_out/r6_79_ab.log; exit 1; }
DGRAD_CFGS=5,6 timeout -k 10 200 python -u tools/bench_dgrad.py > gpurun_out/r6_79_k.log 2>&1 || { tail -20 gpurun_out/r6_79_k.log; exit 1; }
grep -hv amdgpu.ids gpurun_out/r6_79_ab.log; grep -h swiglu gpurun_out/r6_79_k.log
