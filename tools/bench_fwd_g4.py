"""Forward projections y = x W^T (M = 8192, SmolLM3 shapes) on the 4-wave backward kernel in its ROW / ROW form
(gemm_tn cfg 70: 64-deep pair loop, 71: 4-slot ring of 32-deep steps; measured in r5_run33 and removed again,
profiles/r5_gemm_fwd.md — the tool reports them as n/a on the current build) vs the row-contiguous persistent kernel (cfg 60)
and torch.mm on its shipped TunableOp selection. Median of 20, us; max |diff| vs torch.mm.

    python tools/bench_fwd_g4.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts) * 1e3


def main():
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms()
    ops = _ext.ops()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(100):
        a @ a
    del a
    M = 8192
    shapes = [("gate_up", 22016, 2048), ("o_proj", 2048, 2048), ("qkv", 3072, 2048), ("down", 2048, 11008),
              ("lm_head", 128256, 2048)]
    for rep in range(2):
        for name, N, K in shapes:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            ref = torch.mm(x, w.t())
            row = [f"{name:8s}"]
            t = timeit(lambda: torch.mm(x, w.t()))
            row.append(f"blas {t:8.1f}")
            for cfg in (60, 70, 71):
                try:
                    y = ops.gemm_tn(x, w, cfg)
                except RuntimeError:
                    row.append(f"c{cfg}      n/a")
                    continue
                if rep == 0:
                    err = (y.float() - ref.float()).abs().max().item()
                    assert err < 0.05, (name, cfg, err)
                t = timeit(lambda: ops.gemm_tn(x, w, cfg))
                row.append(f"c{cfg} {t:8.1f}")
            print("  ".join(row), flush=True)
            del x, w, ref


if __name__ == "__main__":
    main()
