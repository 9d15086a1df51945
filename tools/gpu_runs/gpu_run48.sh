#!/bin/bash
# SwiGLU fwd/bwd with 1/2/4 vectors in flight per thread and 32-bit index math: tests + kernel timing + bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "swiglu" -x -q --timeout 120 --timeout-method thread > gpurun_out/t48.log 2>&1 || { tail -30 gpurun_out/t48.log; exit 1; }
tail -2 gpurun_out/t48.log
timeout -k 10 120 python - > gpurun_out/s48.log 2>&1 <<'PY' || { tail -20 gpurun_out/s48.log; exit 1; }
import torch, statistics
from llm_fine_tune_distributed_amd.ops import _ext
ops = _ext.ops()
M, I = 8192, 11008
gu = torch.randn(M, 2 * I, device="cuda", dtype=torch.bfloat16)
dy = torch.randn(M, I, device="cuda", dtype=torch.bfloat16)
def t(fn, n=30):
    for _ in range(3): fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    return statistics.median(ts) * 1e3
import os
res = {}
for rnd in range(3):
    for u in ("1", "2", "4"):
        os.environ["SFTAMD_SWIGLU_UNR"] = u
        res.setdefault(u, []).append((t(lambda: ops.swiglu_fwd(gu)), t(lambda: ops.swiglu_bwd(dy, gu))))
for u, v in res.items():
    tf = statistics.median(x[0] for x in v); tb = statistics.median(x[1] for x in v)
    print(f"UNR {u}: swiglu fwd {tf:.1f} us ({3*M*I*2/tf/1e6:.2f} TB/s)  bwd {tb:.1f} us ({5*M*I*2/tb/1e6:.2f} TB/s)")
PY
cat gpurun_out/s48.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>&1 | grep metric > gpurun_out/b48.log || exit 1
python -c "import json; print(json.loads(open('gpurun_out/b48.log').read())['value'])"
