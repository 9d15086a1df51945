#!/bin/bash
# round 6: the input-gradient routing at Llama-3-8B widths — kernel A/B (4-wave 14 vs 8-wave BK-32 5) and the Llama
# step interleaved against SFTAMD_DGRAD_RING8=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_ab.py dgrad l8b_o,l8b_qkv,l8b_gate_up,l8b_down,l8b_lm_head 14,5 --rounds 5 > gpurun_out/r6_56_ab.log 2>&1 || { tail -20 gpurun_out/r6_56_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_56_ab.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2; do
for r in 1 0; do
SFTAMD_DGRAD_RING8=$r timeout -k 10 400 python -u bench.py --model llama3-8b --steps 10 --warmup 3 > gpurun_out/r6_56_l${r}_$i.log 2>&1 || { tail -20 gpurun_out/r6_56_l${r}_$i.log; exit 1; }
echo "llama ring8=$r $i: $(v gpurun_out/r6_56_l${r}_$i.log)"
done
done
