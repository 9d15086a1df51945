#!/bin/bash
# Hybrid data-parallel + split-K wgrad for the partial last round (cfg 1000 + 100 S + variant) on the SmolLM3 shapes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_wgrad.py --only down,qkv,o,gate_up --cfgs 9,10,1210,209,210,410,1209 > gpurun_out/r2_48_micro.log 2>&1 || { tail -20 gpurun_out/r2_48_micro.log; exit 1; }
grep shape gpurun_out/r2_48_micro.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], 'blas', r['blas_ms'], ' '.join(f\"{k[3:-3]}={v}\" for k,v in r.items() if k.endswith('_ms') and k.startswith('cfg')), 'maxerr', max([v for k,v in r.items() if k.endswith('relerr')] or [0]))"
