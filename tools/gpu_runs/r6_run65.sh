#!/bin/bash
# round 6: the SwiGLU down dgrad's wave-tail launch first on a side stream (staggered main rounds) — kernel A/B, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_tail_first.py > gpurun_out/r6_65_k.log 2>&1 || { tail -20 gpurun_out/r6_65_k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_65_k.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for r in 1 0; do
SFTAMD_DGRAD_TAIL_FIRST=$r timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_65_b${r}_$i.log 2>&1 || { tail -20 gpurun_out/r6_65_b${r}_$i.log; exit 1; }
echo "tail_first=$r $i: $(v gpurun_out/r6_65_b${r}_$i.log)"
done
done
