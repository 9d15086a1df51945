"""AdamW flat update (bf16 params + bf16 moments, the training default) with and without stochastic rounding, vs a
pure-bandwidth twin moving the same 14 bytes per parameter (torch copies), at one SmolLM3 layer (80M) and 256M
parameters. Interleaved rounds, median of 10 timed calls."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()


def t(fn, reps=10):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


for n in (80 * 1024 * 1024, 256 * 1024 * 1024):
    p = torch.randn(n, device="cuda").to(torch.bfloat16)
    g = torch.randn(n, device="cuda").to(torch.bfloat16)
    m = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    v = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    coef = torch.ones(1, device="cuda")
    src = torch.empty(4 * n, device="cuda", dtype=torch.bfloat16)
    dst = torch.empty(3 * n, device="cuda", dtype=torch.bfloat16)
    res = {}
    for _ in range(3):
        res.setdefault("sr", []).append(t(lambda: ops.adamw_flat(p, g, None, m, v, coef, 1e-4, 0.9, 0.999, 1e-8, 0.0,
                                                                 0.1, 0.001, 1234, 0)))
        res.setdefault("rne", []).append(t(lambda: ops.adamw_flat(p, g, None, m, v, coef, 1e-4, 0.9, 0.999, 1e-8, 0.0,
                                                                  0.1, 0.001, 0, 0)))
        res.setdefault("copy 8+6 B", []).append(t(lambda: dst.copy_(src[:3 * n]) if False else
                                                  (dst.copy_(src[n:]), None)[1]))
    for k, vals in res.items():
        ms = statistics.median(vals)
        print(f"n={n >> 20}M {k:12s} {ms * 1e3:8.1f} us  {n * 14 / ms / 1e9:.2f} TB/s (14 B/param)", flush=True)
