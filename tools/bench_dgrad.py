"""Input-gradient GEMM microbench: hand-written gfx950 NN dgrad (csrc/gemm_dgrad.hip) vs hipBLASLt (TunableOp),
and the down projection's fused SwiGLU backward vs hipBLASLt + swiglu_bwd. SmolLM3-3B shapes, interleaved rounds.

    python tools/bench_dgrad.py [--tokens 8192]
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


CFGS = [int(c) for c in os.environ.get("DGRAD_CFGS", "7,14").split(",")]


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
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms(verbose=True)
    M = a.tokens
    ops = _ext.ops()
    # dX[M, N] = dy[M, K] . W[K, N]   (W = the projection's [out, in] weight)
    shapes = {"down": (2048, 11008), "o": (2048, 2048), "qkv": (3072, 2048), "gate_up": (22016, 2048)}
    if os.environ.get("DGRAD_SHAPES") == "lm_head":
        shapes = {"lm_head": (128256, 2048), "gate_up": (22016, 2048)}
    res = {}
    data = {}
    for name, (K, N) in shapes.items():
        data[name] = (torch.randn(M, K, device="cuda", dtype=torch.bfloat16),
                      (0.02 * torch.randn(K, N, device="cuda")).to(torch.bfloat16))
    gu = torch.randn(M, 2 * 11008, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.rounds):
        for name, (K, N) in shapes.items():
            dy, w = data[name]
            flop = 2.0 * M * K * N
            r = res.setdefault(name, {"blas": [], **{f"hip{c}": [] for c in CFGS}})
            r["blas"].append(timeit(lambda: torch.mm(dy, w)))
            for cfg in CFGS:
                r[f"hip{cfg}"].append(timeit(lambda: ops.dgrad_gemm(dy, w, None, cfg)))
            r["flop"] = flop
        if "down" not in data:
            continue
        dy, w = data["down"]
        r = res.setdefault("down+swiglu_bwd", {"blas+kernel": [], **{f"fused{c}": [] for c in CFGS}})
        r["blas+kernel"].append(timeit(lambda: ops.swiglu_bwd(torch.mm(dy, w), gu)))
        for cfg in CFGS:
            r[f"fused{cfg}"].append(timeit(lambda: ops.dgrad_gemm(dy, w, gu, cfg)))
        r["flop"] = 2.0 * M * 2048 * 11008
    for name, (K, N) in shapes.items():
        dy, w = data[name]
        ref = torch.mm(dy.float(), w.float())
        for cfg in CFGS:
            e = ((ops.dgrad_gemm(dy, w, None, cfg).float() - ref).norm() / ref.norm()).item()
            res[name][f"relerr{cfg}"] = e
    for name, r in res.items():
        out = {"shape": name, "M": M}
        for k, v in r.items():
            if isinstance(v, list):
                ms = statistics.median(v)
                out[k + "_ms"] = round(ms, 4)
                out[k + "_tflops"] = round(r["flop"] / ms / 1e9, 1)
            elif k.startswith("relerr"):
                out[k] = round(v, 5)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
