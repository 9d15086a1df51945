#!/bin/bash
# round 6: paired weight gradients at several split counts (the _pair_split cost model's check)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_pair.py --pair attn --splits 2,3,4,5,6,8 > gpurun_out/r6_59_attn.log 2>&1 || { tail -20 gpurun_out/r6_59_attn.log; exit 1; }
timeout -k 10 200 python -u tools/bench_pair.py --pair l8b_attn --splits 0,2,3 > gpurun_out/r6_59_l8b.log 2>&1 || { tail -20 gpurun_out/r6_59_l8b.log; exit 1; }
grep -hv amdgpu.ids gpurun_out/r6_59_attn.log gpurun_out/r6_59_l8b.log
