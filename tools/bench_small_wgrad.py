"""Weight-gradient configs for the small SmolLM3 outputs at T = 8192 tokens: o_proj dW[2048, 2048] (64 tiles of
256 x 256) and qkv dW[3072, 2048] (96 tiles). cfg = 1000 H + 100 S + c (csrc/gemm_wgrad.hip: c = 9 / 10 8-wave rings,
12 / 13 4-wave pair / ring; S-way token split, H = hybrid). Median of 20, us; every config checked against cfg 0.

    python tools/bench_small_wgrad.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


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
    ops = _ext.ops()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(100):
        a @ a
    del a
    T = 8192
    for name, N, K, cfgs in (("o_proj", 2048, 2048, (209, 210, 409, 410, 212, 213, 412, 413, 812, 813)),
                             ("qkv", 3072, 2048, (1212, 1213, 210, 212, 213, 312, 313, 412, 413, 812, 813))):
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        ref = (dy.float().t() @ x.float())
        for cfg in cfgs:
            try:
                ops.wgrad_gemm(out, dy, x, False, cfg)
            except RuntimeError as e:
                print(f"{name} cfg {cfg}: n/a ({str(e).splitlines()[0][:80]})", flush=True)
                continue
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(lambda: ops.wgrad_gemm(out, dy, x, False, cfg))
            print(f"{name} cfg {cfg:5d}: {t:7.1f} us  rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
