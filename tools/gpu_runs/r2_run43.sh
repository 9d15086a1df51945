#!/bin/bash
# Stream-K ring wgrad (cfg 2009 / 2010): tests, per-shape microbench vs the ring kernels, bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_43_tests.log 2>&1 || { tail -40 gpurun_out/r2_43_tests.log; exit 1; }
tail -1 gpurun_out/r2_43_tests.log
timeout -k 10 300 python tools/bench_wgrad.py --only gate_up,down,qkv,o --cfgs 10,2010,9,2009,209 > gpurun_out/r2_43_micro.log 2>&1 || { tail -20 gpurun_out/r2_43_micro.log; exit 1; }
grep shape gpurun_out/r2_43_micro.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], 'blas', r['blas_ms'], ' '.join(f\"{k[3:-3]}={v}\" for k,v in r.items() if k.endswith('_ms') and k.startswith('cfg')), 'maxerr', max(v for k,v in r.items() if k.endswith('relerr')))"
for i in 1 2 3; do
  for p in 1 0; do
    SFTAMD_WGRAD_SK=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_43_b$p.log 2>&1 || { tail -30 gpurun_out/r2_43_b$p.log; exit 1; }
    echo "SK=$p $(tail -1 gpurun_out/r2_43_b$p.log | cut -c1-140)"
  done
done
