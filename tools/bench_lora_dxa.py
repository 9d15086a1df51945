"""Micro-benchmark of the LoRA adapter-dx thin GEMM dxa = s dy Bc (csrc/lora.hip dxa_kernel) against torch.addmm
(hipBLASLt) at the SmolLM3-3B LoRA shapes (r = 16 per sub-projection; qkv: 3 adapters, gate_up: 2), interleaved in one
process.

    python tools/bench_lora_dxa.py [--tokens 8192]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=30):
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


ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=int, default=8192)
a = ap.parse_args()
assert _ext.load(), _ext.load_error()
T = a.tokens
print(f"T = {T}")
print("| projection | n | R | addmm us | dense dxa kernel us | block dxa kernel us |")
print("|---|---:|---:|---:|---:|---:|")
# (name, n, r, K, sub-projection row blocks): B_blockdiag has r columns per sub-projection, zero elsewhere
for name, n, r, K, blocks in (("qkv", 3072, 16, 2048, (2048, 512, 512)), ("o", 2048, 16, 2048, (2048,)),
                              ("gate_up", 22016, 16, 2048, (11008, 11008)), ("down", 2048, 16, 11008, (2048,))):
    R = r * len(blocks)
    dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    wide = torch.zeros(n, K + 128, device="cuda", dtype=torch.bfloat16)
    o = [sum(blocks[:i]) for i in range(len(blocks))]
    for i, rows in enumerate(blocks):
        wide[o[i]:o[i] + rows, K + r * i:K + r * (i + 1)] = torch.randn(rows, r, device="cuda") * 0.05
    bc = wide[:, K:K + R]
    c = [r * i for i in range(len(blocks))]
    want = 0.5 * dy.float() @ bc.float()
    out = torch.empty(T, R, device="cuda", dtype=torch.bfloat16)
    t0 = timeit(lambda: torch.addmm(out, dy, bc, beta=0, alpha=0.5))
    t1 = timeit(lambda: _ext.ops().lora_dxa(dy, bc, 0.5))
    t2 = timeit(lambda: _ext.ops().lora_dxa_blocks(dy, bc, o, list(blocks), c, r, 0.5))
    for got in (_ext.ops().lora_dxa(dy, bc, 0.5), _ext.ops().lora_dxa_blocks(dy, bc, o, list(blocks), c, r, 0.5)):
        err = ((got.float() - want).norm() / want.norm()).item()
        assert err < 5e-3, err
    print(f"| {name} | {n} | {R} | {t0 * 1e3:.1f} | {t1 * 1e3:.1f} | {t2 * 1e3:.1f} |", flush=True)
