"""Paired weight-gradient launches (sftamd.wgrad_gemm_pair) at several split counts, interleaved rounds, medians (ms):
the check of ops.fused._pair_split's cost model; --pair layer: the four-problem grid (wgrad_gemm_multi: down + gate_up
+ the next layer's o_proj + qkv) with its leftover split 1..8 ways (ops.fused._multi_split) and, as "pairs", the two
separate pair launches it replaces.

    python tools/bench_pair.py [--pair attn|mlp|l8b_attn|layer] [--splits 0,2,3,4,6] [--rounds 7]

attn = o_proj (2048 x 2048) + qkv (3072 x 2048) at SmolLM3 widths, mlp = down (2048 x 11008) + gate_up (22016 x 2048),
l8b_attn = Llama-3-8B o_proj + qkv; T = 8192 tokens. split 0 = whole rounds + the split leftover (hybrid).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

PAIRS = {  # ((N0, K0), (N1, K1)): out0 [N0, K0] = dy0[T, N0]^T x0[T, K0]
    "attn": ((2048, 2048), (3072, 2048)),
    "mlp": ((2048, 11008), (22016, 2048)),
    "l8b_attn": ((4096, 4096), (6144, 4096)),
}
LAYER = [(2048, 11008), (22016, 2048), (2048, 2048), (3072, 2048)]  # down, gate_up, o_proj, qkv


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
    ap.add_argument("--pair", default="attn", choices=sorted(PAIRS) + ["layer"])
    ap.add_argument("--splits", default="0,2,3,4,6")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=8192)
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    ops = _ext.ops()
    T = a.tokens
    if a.pair == "layer":
        return layer(a, ops, T)
    (N0, K0), (N1, K1) = PAIRS[a.pair]

    def rnd(*s):
        return (0.05 * torch.randn(*s, device="cuda")).to(torch.bfloat16)

    dy0, x0, dy1, x1 = rnd(T, N0), rnd(T, K0), rnd(T, N1), rnd(T, K1)
    out0 = torch.empty(N0, K0, device="cuda", dtype=torch.bfloat16)
    out1 = torch.empty(N1, K1, device="cuda", dtype=torch.bfloat16)
    ref0 = (dy0.float().t() @ x0.float())
    ref1 = (dy1.float().t() @ x1.float())
    splits = [int(s) for s in a.splits.split(",")]
    tiles = (N0 // 256) * (K0 // 256) + (N1 // 256) * (K1 // 256)
    if tiles < 256:
        splits = [s for s in splits if s != 0]  # the hybrid needs at least one whole round

    def run(s):
        ops.wgrad_gemm_pair(out0, dy0, x0, False, None, out1, dy1, x1, False, None, s)

    errs = {}
    for s in splits:
        run(s)
        torch.cuda.synchronize()
        errs[s] = max(((out0.float() - ref0).abs().max() / ref0.abs().max()).item(),
                      ((out1.float() - ref1).abs().max() / ref1.abs().max()).item())
    times = {s: [] for s in splits}
    for r in range(a.rounds):
        order = splits[r % len(splits):] + splits[:r % len(splits)]
        for s in order:
            times[s].append(timeit(lambda: run(s), a.iters))
    rec = {"pair": a.pair, "T": T, "tiles": tiles}
    for s in splits:
        rec[f"split{s}_ms"] = round(statistics.median(times[s]), 4)
        rec[f"split{s}_relerr"] = round(errs[s], 5)
    print(json.dumps(rec), flush=True)


def layer(a, ops, T):
    dys = [(0.05 * torch.randn(T, n, device="cuda")).to(torch.bfloat16) for n, _ in LAYER]
    xs = [(0.05 * torch.randn(T, k, device="cuda")).to(torch.bfloat16) for _, k in LAYER]
    outs = [torch.empty(n, k, device="cuda", dtype=torch.bfloat16) for n, k in LAYER]
    empty = torch.empty(0, device="cuda")
    variants = ["pairs"] + [int(s) for s in a.splits.split(",")]

    def run(v):
        if v == "pairs":
            ops.wgrad_gemm_pair(outs[0], dys[0], xs[0], False, None, outs[1], dys[1], xs[1], False, None, 0)
            ops.wgrad_gemm_pair(outs[2], dys[2], xs[2], False, None, outs[3], dys[3], xs[3], False, None, 3)
        else:
            ops.wgrad_gemm_multi(outs, dys, xs, [0, 0, 0, 0], [empty] * 4, 0, v)

    times = {v: [] for v in variants}
    for r in range(a.rounds):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for v in order:
            times[v].append(timeit(lambda: run(v), a.iters))
    rec = {"pair": "layer", "T": T, "tiles": sum((n // 256) * (k // 256) for n, k in LAYER)}
    for v in variants:
        rec[f"split{v}_ms"] = round(statistics.median(times[v]), 4)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
