#!/bin/bash
# round 6: the MLP weight-gradient pair's time (the calibration of a four-problem launch estimate)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_pair.py --pair mlp --splits 0 > gpurun_out/r6_60_mlp.log 2>&1 || { tail -20 gpurun_out/r6_60_mlp.log; exit 1; }
timeout -k 10 200 python -u tools/bench_pair.py --pair attn --splits 3 > gpurun_out/r6_60_attn.log 2>&1 || { tail -20 gpurun_out/r6_60_attn.log; exit 1; }
timeout -k 10 300 python -u tools/bench_ab.py wgrad gate_up,down,o,qkv 14,1214,414,214 --rounds 5 > gpurun_out/r6_60_ab.log 2>&1 || { tail -20 gpurun_out/r6_60_ab.log; exit 1; }
grep -hv amdgpu.ids gpurun_out/r6_60_mlp.log gpurun_out/r6_60_attn.log gpurun_out/r6_60_ab.log
