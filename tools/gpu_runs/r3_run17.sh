#!/bin/bash
# 4-wave kernels with buffer-descriptor LDS-DMA (SGPR piece offsets): tests, then wgrad / dgrad / forward microbench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py -k "4w or 4wave" \
  > gpurun_out/r3_17_test.log 2>&1 || { tail -40 gpurun_out/r3_17_test.log; exit 1; }
tail -2 gpurun_out/r3_17_test.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 10,9,210,12,13,1213 > gpurun_out/r3_17_wgrad.log 2>&1 || { tail -30 gpurun_out/r3_17_wgrad.log; exit 1; }
grep '^{' gpurun_out/r3_17_wgrad.log | python -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["shape"], {k[:-3]:v for k,v in d.items() if k.endswith("_ms")})'
DGRAD_CFGS=7,12,13 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r3_17_dgrad.log 2>&1 || { tail -30 gpurun_out/r3_17_dgrad.log; exit 1; }
grep '^{' gpurun_out/r3_17_dgrad.log
DGRAD_SHAPES=lm_head DGRAD_CFGS=12,13 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r3_17_dgrad2.log 2>&1 || { tail -30 gpurun_out/r3_17_dgrad2.log; exit 1; }
grep '^{' gpurun_out/r3_17_dgrad2.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 12,50,60,61 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048 > gpurun_out/r3_17_tn.log 2>&1 || { tail -30 gpurun_out/r3_17_tn.log; exit 1; }
cat gpurun_out/r3_17_tn.log
