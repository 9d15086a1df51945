"""Sweep the forward-layout GEMM variants (cfg) on the big SmolLM3 shapes; GROUP from env."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from llm_fine_tune_distributed_amd.ops import _ext
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
assert _ext.load(), _ext.load_error()
enable_tuned_gemms()
ops = _ext.ops()
M = 8192
def timeit(fn, n=15):
    for _ in range(3): fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    return statistics.median(ts)
out = [f"GROUP={os.environ.get('SFTAMD_TN_GROUP', '8')}"]
for name, N, K in [("gate_up", 22016, 2048), ("down", 2048, 11008), ("lm_head", 128256, 2048)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    fl = 2.0 * M * N * K
    r = [name, f"blas {fl / timeit(lambda: torch.nn.functional.linear(x, w)) / 1e9:.0f}"]
    for cfg in (2, 4):
        r.append(f"cfg{cfg} {fl / timeit(lambda: ops.gemm_tn(x, w, cfg)) / 1e9:.0f}")
    out.append(" ".join(r))
print(" | ".join(out), flush=True)
