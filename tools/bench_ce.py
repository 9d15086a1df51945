#!/usr/bin/env python3
"""Fused cross-entropy kernel (csrc/cross_entropy.hip) at the bench shape: M = 8192 rows x V = 128256 bf16 logits,
loss / lse / entropy / accuracy + the in-place bf16 gradient. Prints time per call and the HBM rate
(2 reads + 1 write of the logits)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    base = (torch.randn(a.rows, a.vocab, device=dev, generator=g) * 2).to(torch.bfloat16)
    labels = torch.randint(0, a.vocab, (a.rows,), device=dev, generator=g)
    inv = torch.tensor([1.0 / a.rows], device=dev)
    work = base.clone()
    out = {}
    for write_grad in (False, True):
        for _ in range(3):
            work.copy_(base)
            _ext.ops().ce_fwd(work, labels, inv, write_grad)
        ts = []
        for _ in range(a.iters):
            work.copy_(base)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            _ext.ops().ce_fwd(work, labels, inv, write_grad)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ms = sorted(ts)[len(ts) // 2]
        nbytes = a.rows * a.vocab * 2 * (3 if write_grad else 1)
        out["grad" if write_grad else "stats"] = {"ms": round(ms, 4), "TB_s": round(nbytes / ms / 1e9, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
