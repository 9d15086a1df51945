"""Does a partial last round cost a full round? wgrad (4-wave, cfg 14) time vs tile count at K = 2048, T = 8192:
quantised grids would step at multiples of 256 tiles, power-bound ones scale with the tile count."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
T, K = 8192, 2048
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
res = {}
Ns = [256 * n for n in (32, 48, 64, 72, 80, 86, 88, 96, 104, 128)]
dys = {N: torch.randn(T, N, device="cuda", dtype=torch.bfloat16) for N in Ns}
outs = {N: torch.empty(N, K, device="cuda", dtype=torch.bfloat16) for N in Ns}
for rnd in range(5):
    for N in Ns:
        f = lambda: ops.wgrad_gemm(outs[N], dys[N], x, False, 14)
        f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        res.setdefault(N, []).append(s.elapsed_time(e) / 10)
for N in Ns:
    tiles = (N // 256) * (K // 256)
    t = statistics.median(res[N])
    print(f"tiles {tiles:5d} rounds {tiles / 256:5.2f}  {t:.4f} ms  {t / tiles * 256:.4f} ms per 256 tiles", flush=True)
