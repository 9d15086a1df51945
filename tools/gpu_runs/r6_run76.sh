#!/bin/bash
# round 6: the SwiGLU down dgrad's partial 6th round unsplit (SFTAMD_DGRAD_TAIL=0: 96 whole tiles at 37.5 % occupancy)
# vs the 256 x 128 half-tile launch (default) — kernel and step, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
for t in 2 0; do
SFTAMD_DGRAD_TAIL=$t DGRAD_CFGS=5 timeout -k 10 200 python -u tools/bench_dgrad.py > gpurun_out/r6_76_k${t}_$i.log 2>&1 || { tail -20 gpurun_out/r6_76_k${t}_$i.log; exit 1; }
echo "tail=$t $i: $(grep -h 'swiglu' gpurun_out/r6_76_k${t}_$i.log | grep -o '"fused5_ms": [0-9.]*')  $(grep -h '"shape": "down"' gpurun_out/r6_76_k${t}_$i.log | grep -o '"hip5_ms": [0-9.]*')"
done
done
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for t in 2 0; do
SFTAMD_DGRAD_TAIL=$t timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_76_b${t}_$i.log 2>&1 || { tail -20 gpurun_out/r6_76_b${t}_$i.log; exit 1; }
echo "step tail=$t $i: $(v gpurun_out/r6_76_b${t}_$i.log)"
done
done
