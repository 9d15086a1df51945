"""AdamW flat-update bandwidth on 1x MI355X (csrc/optim.hip adamw_kernel): bf16 params + bf16 moments with stochastic
rounding (the training default) against round-to-nearest (sr_seed = 0: same bytes, no hashing) and fp32 moments —
whether the update is HBM- or VALU-bound. Interleaved rounds, median of 10 timed calls each.

    python tools/bench_adamw.py [N elements, default 256M]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256 * 1024 * 1024
p = torch.randn(n, device="cuda").to(torch.bfloat16)
g = torch.randn(n, device="cuda").to(torch.bfloat16)
coef = torch.ones(1, device="cuda")
state = {dt: (torch.zeros(n, device="cuda", dtype=dt), torch.zeros(n, device="cuda", dtype=dt))
         for dt in (torch.float32, torch.bfloat16)}


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


# (round 5, r5_run14: launch shapes of 2 / 4 vectors of 8 per thread step x 1024 / 2048 / 4096 blocks; 4 x 2048, now
# the default, was fastest for bf16 moments: 759 vs 822 us with SR)
res = {}
for rnd in range(3):
    for dt, (m, v) in state.items():
        for sr in (1234, 0):
            ms = t(lambda: ops.adamw_flat(p, g, None, m, v, coef, 1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, sr, 0))
            res.setdefault((str(dt).replace("torch.", ""), "SR" if sr else "RN"), []).append(ms)
for (dt, sr), v in res.items():
    ms = statistics.median(v)
    bpp = 22 if dt == "float32" else 14
    print(f"moments {dt:8s} {sr}: {ms * 1e3:8.1f} us  {n * bpp / ms / 1e9:.2f} TB/s", flush=True)
