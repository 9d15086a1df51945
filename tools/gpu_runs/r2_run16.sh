#!/bin/bash
# Round 2: dgrad tile configs (256x256 vs 256x128) correctness + microbench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k dgrad --timeout 120 --timeout-method thread > gpurun_out/r2_16_tests.log 2>&1 || { tail -40 gpurun_out/r2_16_tests.log; exit 1; }
tail -1 gpurun_out/r2_16_tests.log
DGRAD_CFGS=1,5,7 timeout -k 10 300 python tools/bench_dgrad.py > gpurun_out/r2_16_dgrad.log 2>&1 || { tail -20 gpurun_out/r2_16_dgrad.log; exit 1; }
grep shape gpurun_out/r2_16_dgrad.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], {k[:-3]: v for k, v in r.items() if k.endswith('_ms')})"
