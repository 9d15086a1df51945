#!/bin/bash
# qkv+RoPE forward GEMM wave-quantisation tail (SFTAMD_TN_TAIL): tests, microbench, bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "tn_rope or model" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_56_tests.log 2>&1 || { tail -40 gpurun_out/r2_56_tests.log; exit 1; }
tail -1 gpurun_out/r2_56_tests.log
cat > /tmp/tnbench.py <<'PY'
import os, statistics, sys, torch
sys.path.insert(0, os.getcwd())
from llm_fine_tune_distributed_amd.ops import _ext
assert _ext.load()
ops = _ext.ops()
M, K, N = 8192, 2048, 3072
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
cs = torch.rand(M, 64, device="cuda"); sn = torch.rand(M, 64, device="cuda")
def t(fn, n=50):
    for _ in range(5): fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    return statistics.median(ts)
res = {}
for r in range(3):
    for tail in ("0", "1"):
        os.environ["SFTAMD_TN_TAIL"] = tail
        res.setdefault(tail, []).append(t(lambda: ops.gemm_tn_rope(x, w, cs, sn, 2560, 11)))
for k, v in res.items():
    print(f"qkv+rope tail={k}: {statistics.median(v)*1e3:.1f} us")
PY
timeout -k 10 300 python /tmp/tnbench.py > gpurun_out/r2_56_micro.log 2>&1 || { tail -20 gpurun_out/r2_56_micro.log; exit 1; }
cat gpurun_out/r2_56_micro.log
for i in 1 2 3; do
  for p in 1 0; do
    SFTAMD_TN_TAIL=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_56_b$p.log 2>&1 || { tail -30 gpurun_out/r2_56_b$p.log; exit 1; }
    echo "TN_TAIL=$p $(tail -1 gpurun_out/r2_56_b$p.log | cut -c1-120)"
  done
done
