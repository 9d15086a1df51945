#!/bin/bash
# hybrid split-K with whole tiles on the first dispatch rounds (block-index classes): tests, dgrad M = 10240,
# wgrad hybrid variants at T = 8192, then the recipe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py -k "wgrad or dgrad or 4w" > gpurun_out/r3_24_test.log 2>&1 || { tail -30 gpurun_out/r3_24_test.log; exit 1; }
tail -2 gpurun_out/r3_24_test.log
DGRAD_SHAPES=lm_head DGRAD_CFGS=13 timeout -k 10 300 python -u tools/bench_dgrad.py --tokens 10240 > gpurun_out/r3_24_dg2.log 2>&1 || { tail -20 gpurun_out/r3_24_dg2.log; exit 1; }
grep '^{' gpurun_out/r3_24_dg2.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 10,9,13,1213,1313,1310,1309 --only gate_up,down > gpurun_out/r3_24_wg.log 2>&1 || { tail -30 gpurun_out/r3_24_wg.log; exit 1; }
grep '^{' gpurun_out/r3_24_wg.log | python -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["shape"], {k[:-3]:v for k,v in d.items() if k.endswith("_ms")})'
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_24_rec.log 2>&1 || { tail -20 gpurun_out/r3_24_rec.log; exit 1; }
grep '"metric"' gpurun_out/r3_24_rec.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rec", d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["final_eval_loss"])'
