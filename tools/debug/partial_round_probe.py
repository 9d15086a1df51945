"""Unsplit partial rounds vs token-split pieces for the weight-gradient grids that are not whole rounds: the o_proj +
qkv pair alone (160 tiles: one partial round unsplit vs every tile split 3 ways) and the lm_head (4008 tiles: 15
rounds + 168 tiles, unsplit cfg 14 vs the hybrid 1214). ms, interleaved medians, T = 8192."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    assert _ext.load(), _ext.load_error()
    ops = _ext.ops()
    T = 8192

    def rnd(*s):
        return (0.05 * torch.randn(*s, device="cuda")).to(torch.bfloat16)

    empty = torch.empty(0, device="cuda")
    shapes = [(2048, 2048), (3072, 2048)]
    dys, xs = [rnd(T, n) for n, _ in shapes], [rnd(T, k) for _, k in shapes]
    outs = [torch.empty(n, k, device="cuda", dtype=torch.bfloat16) for n, k in shapes]
    var = {"attn_unsplit": lambda: ops.wgrad_gemm_multi(outs, dys, xs, [0, 0], [empty] * 2, 0, 1),
           "attn_split3": lambda: ops.wgrad_gemm_multi(outs, dys, xs, [0, 0], [empty] * 2, 3, 0)}
    dl, xl = rnd(T, 128256), rnd(T, 2048)
    ol = torch.empty(128256, 2048, device="cuda", dtype=torch.bfloat16)
    var["lm_head_14"] = lambda: ops.wgrad_gemm(ol, dl, xl, False, 14)
    var["lm_head_1214"] = lambda: ops.wgrad_gemm(ol, dl, xl, False, 1214)
    times = {k: [] for k in var}
    names = list(var)
    for r in range(7):
        for k in names[r % len(names):] + names[:r % len(names)]:
            times[k].append(timeit(var[k]))
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in times.items()}), flush=True)


if __name__ == "__main__":
    main()
