"""Weight-gradient GEMM microbench: hand-written gfx950 kernel vs tuned hipBLASLt/rocBLAS (TunableOp).

    python tools/bench_wgrad.py [--tokens 8192]
Shapes are the SmolLM3-3B training wgrads: dW[N,K] = dy[T,N]^T x[T,K].
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--cfgs", default="14,1214,10")
    ap.add_argument("--only", default="")
    ap.add_argument("--no-blas", action="store_true")
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms(verbose=True)
    T = a.tokens
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (22016, 2048), "down": (2048, 11008),
              "lm_head": (128256, 2048)}
    for name, (N, K) in shapes.items():
        if a.only and name not in a.only.split(","):
            continue
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * T * N * K
        rec = {"shape": name, "T": T, "N": N, "K": K}
        ms = timeit(lambda: torch.mm(dy.t(), x, out=out), iters=2 if a.no_blas else 20)
        ref = out.float().clone()
        rec["blas_ms"] = round(ms, 4)
        rec["blas_tflops"] = round(flop / ms / 1e9, 1)
        for cfg in [int(c) for c in a.cfgs.split(",")]:
            if cfg % 100 in (1, 3, 7, 8, 10) and (N % 256 or K % 256):
                continue
            if N % 256 or K % 128:
                continue
            try:
                ms = timeit(lambda: _ext.ops().wgrad_gemm(out, dy, x, False, cfg))
            except RuntimeError as e:  # shape not supported by this variant
                rec[f"cfg{cfg}"] = str(e).split(":")[-1].strip()[:60]
                continue
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            rec[f"cfg{cfg}_ms"] = round(ms, 4)
            rec[f"cfg{cfg}_tflops"] = round(flop / ms / 1e9, 1)
            rec[f"cfg{cfg}_relerr"] = round(err, 5)
        print(json.dumps(rec), flush=True)
        del dy, x, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
