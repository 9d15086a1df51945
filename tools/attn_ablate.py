"""Timing-only ablations of the attention forward v3 (SFTAMD_ATTN_DIAG bits, wrong results)."""
import math, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from llm_fine_tune_distributed_amd.ops import _ext
assert _ext.load()
B, T, NQ, NKV, D = 16, 512, 16, 4, 128
M = B * T
cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device="cuda")
qkv = torch.randn(M, (NQ + 2 * NKV) * D, device="cuda", dtype=torch.bfloat16)
ops = _ext.ops()
def timeit(fn, n=30):
    for _ in range(3): fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    return statistics.median(ts)
os.environ["SFTAMD_ATTN_IMPL"] = "3"
res = {}
for rnd in range(3):
    for d in ("0", "1", "2", "4", "8", "12", "15"):
        os.environ["SFTAMD_ATTN_DIAG"] = d
        res.setdefault(d, []).append(timeit(lambda: ops.flash_fwd(qkv, cu, T, NQ, NKV, D, 1 / math.sqrt(D), True)))
names = {"0": "full", "1": "no loop loads", "2": "no softmax", "4": "no PV mfma", "8": "no QK mfma", "12": "no mfma", "15": "nothing"}
for d, v in res.items():
    print(f"DIAG {d:>2} ({names[d]}): {statistics.median(v) * 1e3:.1f} us")
