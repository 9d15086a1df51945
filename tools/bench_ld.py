"""Does a power-of-two row pitch cost the GEMMs? The SmolLM3 activations are [tokens, 2048] bf16 = 4 KiB rows: every row
of a tile starts at the same address modulo 4 KiB. Times the same products with the operands' row pitch padded (a
strided view into a wider buffer), same data and shapes, M = 8192:

  forward  y = x W^T     (gate_up 22016 x 2048, o 2048 x 2048): torch.mm (TunableOp selections loaded) and the
                          row-contiguous persistent kernel (gemm_tn cfg 60), x pitch 2048 / 2080 / 2112 / 2176
  dgrad    dX = dY W      (gate_up, o_proj): the 4-wave kernel, the 2048-wide operands' pitch +0 / +64 / +128

    python tools/bench_ld.py
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


def padded(t, ld):
    if ld == t.shape[1]:
        return t
    buf = torch.empty(t.shape[0], ld, device=t.device, dtype=t.dtype)
    buf[:, :t.shape[1]] = t
    return buf[:, :t.shape[1]]


def main():
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms()
    ops = _ext.ops()
    M = 8192
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(100):  # clocks up first
        a @ a
    for name, N, K in (("gate_up", 22016, 2048), ("o_proj", 2048, 2048), ("qkv", 3072, 2048)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        for ld in (K, K + 32, K + 64, K + 128):
            xp = padded(x, ld)
            tb = timeit(lambda: torch.mm(xp, w.t()))
            th = timeit(lambda: ops.gemm_tn(xp, w, 60))
            print(f"fwd {name:8s} x pitch {ld:5d}: torch.mm {tb:8.1f} us   gemm_tn cfg60 {th:8.1f} us", flush=True)
    # input gradients: gate_up (dY [8192, 22016] . W [22016, 2048]: W rows are 4 KiB) and o_proj (dY and W both
    # [.., 2048]: 4 KiB rows) on the 4-wave kernel, the 2048-wide operands padded
    for name, N, K in (("gate_up", 22016, 2048), ("o_proj", 2048, 2048)):
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        for ld in (K, K + 64, K + 128):
            wp = padded(w, ld)
            dyp = padded(dy, N + ld - K) if N == 2048 else dy
            td = timeit(lambda: ops.dgrad_gemm(dyp, wp, None, 13 if N > 4096 else 12))
            print(f"dgrad {name:8s} pitch +{ld - K:3d}: {td:8.1f} us", flush=True)

if __name__ == "__main__":
    main()
