"""Micro-benchmark of the forward-layout HIP GEMM (csrc/gemm_tn.hip) against hipBLASLt/rocBLAS
(torch linear through TunableOp with the shipped MI355X selections), at the SmolLM3-3B training
shapes (M = 16 x 512 tokens). Fused variants are timed against their unfused twins
(BLAS GEMM + the separate SwiGLU / RoPE kernel). Interleaved in one process (CDNA guide rule 24).

    python tools/bench_gemm_tn.py [--m 8192]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=8192)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--cfgs", default="0,2,5,11,60,61", help="gemm_tn configurations to time")
ap.add_argument("--shapes", default="", help="name:N:K,... instead of the SmolLM3 projection shapes")
ap.add_argument("--plain-only", action="store_true", help="skip the fused-epilogue section")
ap.add_argument("--fused-cfgs", default="", help="time only gemm_tn_swiglu / gemm_tn_rope at these cfgs vs their unfused "
                                                  "twins (skips the plain table)")
a = ap.parse_args()
assert _ext.load(), _ext.load_error()
enable_tuned_gemms()
ops = _ext.ops()
M = a.m
torch.manual_seed(0)


def timeit(fn, n=a.iters):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def rel(a_, b_):
    return ((a_.float() - b_.float()).norm() / b_.float().norm()).item()


print(f"M = {M}")
if a.fused_cfgs:
    FC = [int(c) for c in a.fused_cfgs.split(",")]
    K, I = 2048, 11008
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    wgu = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16) * 0.02
    gu_ref = torch.nn.functional.linear(x, wgu)
    t0 = timeit(lambda: ops.swiglu_fwd(torch.nn.functional.linear(x, wgu)))
    tb = timeit(lambda: torch.nn.functional.linear(x, wgu))
    row = [f"blas {tb:.3f} + swiglu kernel = {t0:.3f}"]
    for c in FC:
        gu, act = ops.gemm_tn_swiglu(x, wgu, c)
        assert rel(gu, gu_ref) < 1e-2, c
        row.append(f"cfg {c} {timeit(lambda: ops.gemm_tn_swiglu(x, wgu, c)):.3f}")
    print("gate_up + SwiGLU (ms): " + ", ".join(row), flush=True)
    nq, nkv, D = 16, 4, 128
    wq = torch.randn((nq + 2 * nkv) * D, K, device="cuda", dtype=torch.bfloat16) * 0.02
    pos = torch.arange(512, device="cuda").repeat(M // 512).float()
    inv = 1.0 / (2e6 ** (torch.arange(0, D, 2, device="cuda").float() / D))
    fr = pos[:, None] * inv[None, :]
    cs, sn = fr.cos().contiguous(), fr.sin().contiguous()

    def unf():
        q = torch.nn.functional.linear(x, wq)
        ops.rope_(q, cs, sn, nq, nkv, D, False)
        return q
    qr = unf()
    row = [f"blas + rope kernel {timeit(unf):.3f}"]
    for c in FC:
        assert rel(ops.gemm_tn_rope(x, wq, cs, sn, (nq + nkv) * D, c), qr) < 1e-2, c
        row.append(f"cfg {c} {timeit(lambda: ops.gemm_tn_rope(x, wq, cs, sn, (nq + nkv) * D, c)):.3f}")
    print("qkv + RoPE (ms): " + ", ".join(row), flush=True)
    sys.exit(0)
CFGS = [int(c) for c in a.cfgs.split(",")]
print("| shape | N | K | blas ms (TF/s) | " + " | ".join(f"cfg {c}" for c in CFGS) + " | max rel err |")
print("|---|---:|---:|---:|" + "---:|" * len(CFGS) + "---:|")
SHAPES = ([(f.split(":")[0], int(f.split(":")[1]), int(f.split(":")[2])) for f in a.shapes.split(",")] if a.shapes else
          [("qkv", 3072, 2048), ("o", 2048, 2048), ("gate_up", 22016, 2048), ("down", 2048, 11008),
           ("lm_head", 128256, 2048)])
for name, N, K in SHAPES:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    fl = 2.0 * M * N * K
    ref = torch.nn.functional.linear(x, w)
    row = [name, str(N), str(K)]
    t = timeit(lambda: torch.nn.functional.linear(x, w))
    row.append(f"{t:.3f} ({fl / t / 1e9:.0f})")
    err = 0.0
    for cfg in CFGS:
        c = ops.gemm_tn(x, w, cfg)
        err = max(err, rel(c, ref))
        t = timeit(lambda: ops.gemm_tn(x, w, cfg))
        row.append(f"{t:.3f} ({fl / t / 1e9:.0f})")
    row.append(f"{err:.4f}")
    print("| " + " | ".join(row) + " |", flush=True)
    del x, w, ref

if a.plain_only:
    sys.exit(0)
# fused epilogues vs unfused twins
K, I = 2048, 11008
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
wgu = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16) * 0.02
gu_ref = torch.nn.functional.linear(x, wgu)
act_ref = ops.swiglu_fwd(gu_ref)
gu, act = ops.gemm_tn_swiglu(x, wgu)
print(f"\nswiglu fused: gu rel err {rel(gu, gu_ref):.4f}, act rel err {rel(act, act_ref):.4f}")
t0 = timeit(lambda: ops.swiglu_fwd(torch.nn.functional.linear(x, wgu)))
t1 = timeit(lambda: ops.gemm_tn_swiglu(x, wgu))
print(f"gate_up + SwiGLU: blas + kernel {t0:.3f} ms, fused {t1:.3f} ms ({(t0 - t1) * 1e3:.0f} us saved per layer)")

nq, nkv, D = 16, 4, 128
wq = torch.randn((nq + 2 * nkv) * D, K, device="cuda", dtype=torch.bfloat16) * 0.02
pos = torch.arange(512, device="cuda").repeat(M // 512).float()
inv = 1.0 / (2e6 ** (torch.arange(0, D, 2, device="cuda").float() / D))
fr = pos[:, None] * inv[None, :]
cs, sn = fr.cos().contiguous(), fr.sin().contiguous()


def unfused():
    q = torch.nn.functional.linear(x, wq)
    ops.rope_(q, cs, sn, nq, nkv, D, False)
    return q


qr = unfused()
t0 = timeit(unfused)
parts = [f"blas + kernel {t0:.3f} ms"]
for cfg in (0, 2, 5, 11, 60, 61):
    qf = ops.gemm_tn_rope(x, wq, cs, sn, (nq + nkv) * D, cfg)
    t = timeit(lambda: ops.gemm_tn_rope(x, wq, cs, sn, (nq + nkv) * D, cfg))
    parts.append(f"cfg{cfg} {t:.3f} ms (rel err {rel(qf, qr):.4f})")
print("qkv + RoPE: " + ", ".join(parts))
