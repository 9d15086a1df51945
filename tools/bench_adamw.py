"""AdamW flat-update bandwidth on 1x MI355X: launch shapes (SFTAMD_ADAM_UNR x SFTAMD_ADAM_BLOCKS), fp32 and bf16
moments, stochastic rounding on (the training default). Interleaved rounds, median of 10 timed calls each."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
n = int(os.environ.get("N", 256 * 1024 * 1024))
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


cfgs = [(u, b) for u in ("1", "2") for b in ("1024", "2048", "4096", "8192")]
res = {}
for rnd in range(3):
    for dt, (m, v) in state.items():
        for u, b in cfgs:
            os.environ["SFTAMD_ADAM_UNR"], os.environ["SFTAMD_ADAM_BLOCKS"] = u, b
            ms = t(lambda: ops.adamw_flat(p, g, None, m, v, coef, 1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, 1234, 0))
            res.setdefault((str(dt), u, b), []).append(ms)
for (dt, u, b), v in res.items():
    ms = statistics.median(v)
    bpp = 22 if "float32" in dt else 14
    print(f"{dt:15s} UNR {u} blocks {b:>5s}: {ms * 1e3:8.1f} us  {n * bpp / ms / 1e9:.2f} TB/s")
