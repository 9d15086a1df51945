#!/bin/bash
# Round 2: hybrid data-parallel + split-K wgrad: correctness + microbench on every SmolLM3 wgrad shape.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/r2_05_tests.log 2>&1 || { tail -40 gpurun_out/r2_05_tests.log; exit 1; }
tail -1 gpurun_out/r2_05_tests.log
timeout -k 10 400 python tools/bench_wgrad.py --cfgs 9,10,209,409,210,310,1209,1309,1409,1210,1310,1410 > gpurun_out/r2_05_wgrad.log 2>&1 || { tail -20 gpurun_out/r2_05_wgrad.log; exit 1; }
timeout -k 10 400 python tools/bench_wgrad.py --tokens 4096 --no-blas --cfgs 9,10,209,409,210,310,1209,1309,1210,1310 > gpurun_out/r2_05_wgrad4k.log 2>&1 || { tail -20 gpurun_out/r2_05_wgrad4k.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r2_05_wgrad.log", "gpurun_out/r2_05_wgrad4k.log"):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            ms = {k[3:-3]: v for k, v in r.items() if k.endswith("_ms")}
            best = min(ms, key=ms.get)
            print(r["shape"], r["T"], "best", best, ms[best], " ".join(f"{k}={v}" for k, v in sorted(ms.items(), key=lambda t: t[1])[:5]))
PY
