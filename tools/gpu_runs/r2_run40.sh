#!/bin/bash
# dgrad wave-quantisation tail split (SFTAMD_DGRAD_TAIL): tests, down dgrad+SwiGLU microbench, bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_40_tests.log 2>&1 || { tail -40 gpurun_out/r2_40_tests.log; exit 1; }
tail -1 gpurun_out/r2_40_tests.log
cat > /tmp/tailbench.py <<'PY'
import os, statistics, sys, torch
sys.path.insert(0, os.getcwd())
from llm_fine_tune_distributed_amd.ops import _ext
assert _ext.load()
ops = _ext.ops()
M, K, N = 8192, 2048, 11008
dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = (0.02 * torch.randn(K, N, device="cuda")).to(torch.bfloat16)
gu = torch.randn(M, 2 * N, device="cuda", dtype=torch.bfloat16)
def t(fn, n=30):
    for _ in range(5): fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    return statistics.median(ts)
res = {}
for r in range(3):
    for cfg in (7, 0):
        for tail in ("0", "2", "3"):
            os.environ["SFTAMD_DGRAD_TAIL"] = tail
            res.setdefault((cfg, tail), []).append(t(lambda: ops.dgrad_gemm(dy, w, gu, cfg)))
for k, v in res.items():
    print(f"down dgrad+swiglu cfg {k[0]} tail {k[1]}: {statistics.median(v)*1e3:.1f} us")
PY
timeout -k 10 300 python /tmp/tailbench.py > gpurun_out/r2_40_micro.log 2>&1 || { tail -20 gpurun_out/r2_40_micro.log; exit 1; }
cat gpurun_out/r2_40_micro.log
for i in 1 2 3; do
  for p in 2 0; do
    SFTAMD_DGRAD_TAIL=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_40_b$p.log 2>&1 || { tail -30 gpurun_out/r2_40_b$p.log; exit 1; }
    echo "TAIL=$p $(tail -1 gpurun_out/r2_40_b$p.log | cut -c1-140)"
  done
done
