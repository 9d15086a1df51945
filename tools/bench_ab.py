"""Interleaved A/B of backward GEMM variants: every round times every (shape, variant) once, in a rotated order, so
clock drift and order effects spread evenly over the variants; medians over the rounds (ms) and the max relative
error against the first variant.

    python tools/bench_ab.py wgrad gate_up 14,1214,15,1215 [--rounds 7]
    python tools/bench_ab.py dgrad gate_up 14,15,16
    python tools/bench_ab.py wgrad lm_head 10,1214 --rounds 5

wgrad: dW[N, K] = dy[T, N]^T x[T, K] (sftamd.wgrad_gemm cfg); fwd: y[T, N] = x[T, K] W[N, K]^T (sftamd.gemm_tn cfg); dgrad: dX[T, N] = dy[T, K] W[K, N] (sftamd.dgrad_gemm cfg;
'blas' = torch.mm on the TunableOp selection; 'delta' = dgrad_gemm_delta). SmolLM3-3B shapes at T = 8192 tokens;
Llama-3-8B ones as l8b_qkv, l8b_o, l8b_gate_up, l8b_down, l8b_lm_head.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402

WGRAD = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (22016, 2048), "down": (2048, 11008),
         "lm_head": (128256, 2048)}
DGRAD = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (22016, 2048), "down": (2048, 11008),
         "lm_head": (128256, 2048)}  # (K, N): dX[T, N] = dy[T, K] W[K, N]
# Llama-3-8B widths (hidden 4096, 32 q / 8 kv heads x 128, intermediate 14336): the same layouts, "l8b_" names
WGRAD.update({"l8b_qkv": (6144, 4096), "l8b_o": (4096, 4096), "l8b_gate_up": (28672, 4096),
              "l8b_down": (4096, 14336), "l8b_lm_head": (128256, 4096)})
DGRAD.update({k: v for k, v in WGRAD.items() if k.startswith("l8b_")})


def timeit(fn, iters):
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
    ap.add_argument("kind", choices=["wgrad", "dgrad", "fwd"])
    ap.add_argument("shapes")
    ap.add_argument("variants")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms()
    ops = _ext.ops()
    T = a.tokens
    variants = a.variants.split(",")
    for name in a.shapes.split(","):
        if a.kind == "wgrad":
            N, K = WGRAD[name]
            dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)

            def run(v):
                if v == "blas":
                    torch.mm(dy.t(), x, out=out)
                else:
                    ops.wgrad_gemm(out, dy, x, False, int(v))
                return out
        elif a.kind == "fwd":
            N, K = WGRAD[name]  # y[T, N] = x[T, K] W[N, K]^T
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
            hold = [None]

            def run(v):
                hold[0] = torch.mm(x, w.t()) if v == "blas" else ops.gemm_tn(x, w, int(v))
                return hold[0]
        else:
            K, N = DGRAD[name]
            dy = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            w = (0.02 * torch.randn(K, N, device="cuda")).to(torch.bfloat16)
            holder = [None]

            a_out = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)

            def run(v):  # 'delta': cfg 14 with flash attention's delta in the epilogue (dgrad_gemm_delta)
                if v == "blas":
                    holder[0] = torch.mm(dy, w)
                elif v == "delta":
                    holder[0] = ops.dgrad_gemm_delta(dy, w, a_out)[0]
                else:
                    holder[0] = ops.dgrad_gemm(dy, w, None, int(v))
                return holder[0]
        ref = run(variants[0]).float().clone()
        errs = {}
        for v in variants:
            y = run(v).float()
            errs[v] = ((y - ref).abs().max() / ref.abs().max()).item()
        times = {v: [] for v in variants}
        for r in range(a.rounds):
            order = variants[r % len(variants):] + variants[:r % len(variants)]
            for v in order:
                times[v].append(timeit(lambda: run(v), a.iters))
        rec = {"kind": a.kind, "shape": name, "T": T}
        for v in variants:
            rec[f"{v}_ms"] = round(statistics.median(times[v]), 4)
            rec[f"{v}_relerr"] = round(errs[v], 5)
        print(json.dumps(rec), flush=True)
        del ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
