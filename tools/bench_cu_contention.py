"""What the GEMM grids lose when some CUs are held by other work — the situation of an RCCL collective overlapped with
the backward at N > 1: its channel blocks sit on CUs, and a kernel whose grid is exactly one round of 256 one-per-CU
workgroups (the 4-wave ring holds a CU's whole register file) then needs a second round.

    python tools/bench_cu_contention.py [--held 0,8,16,32] [--iters 20]

For each held-CU count C, `sftamd.cu_hog(sink, C, ...)` occupies C CUs on a side stream (one workgroup per CU, sleeping)
while the op is timed on the main stream; ms per call, SmolLM3 shapes at T = 8192 tokens.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--held", default="0,8,16,32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=8192)
    a = ap.parse_args()
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms()
    ops = _ext.ops()
    T = a.tokens
    dev = "cuda"

    def rnd(*s):
        return (0.05 * torch.randn(*s, device=dev)).to(torch.bfloat16)

    x2k, x11k = rnd(T, 2048), rnd(T, 11008)
    dy2k, dy3k, dy22k, dy11k = rnd(T, 2048), rnd(T, 3072), rnd(T, 22016), rnd(T, 11008)
    w_o, w_qkv, w_gu, w_d = rnd(2048, 2048), rnd(3072, 2048), rnd(22016, 2048), rnd(2048, 11008)
    out = {k: torch.empty(s, device=dev, dtype=torch.bfloat16)
           for k, s in (("o", (2048, 2048)), ("qkv", (3072, 2048)), ("gu", (22016, 2048)), ("d", (2048, 11008)))}
    cases = {
        "wgrad o 414": lambda: ops.wgrad_gemm(out["o"], dy2k, x2k, False, 414),
        "wgrad o 214": lambda: ops.wgrad_gemm(out["o"], dy2k, x2k, False, 214),
        "wgrad qkv 214": lambda: ops.wgrad_gemm(out["qkv"], dy3k, x2k, False, 214),
        "wgrad gate_up 14": lambda: ops.wgrad_gemm(out["gu"], dy22k, x2k, False, 14),
        "wgrad down 1214": lambda: ops.wgrad_gemm(out["d"], dy2k, x11k, False, 1214),
        "dgrad o 14": lambda: ops.dgrad_gemm(dy2k, w_o, None, 14),
        "dgrad qkv 14": lambda: ops.dgrad_gemm(dy3k, w_qkv, None, 14),
        "dgrad gate_up 14": lambda: ops.dgrad_gemm(dy22k, w_gu, None, 14),
        "fwd o blas": lambda: torch.mm(x2k, w_o.t()),
        "fwd gate_up blas": lambda: torch.mm(x2k, w_gu.t()),
        "fwd down blas": lambda: torch.mm(x11k, w_d.t()),
    }
    side = torch.cuda.Stream()
    sink = torch.zeros(256, device=dev, dtype=torch.int32)
    held = [int(c) for c in a.held.split(",")]
    for name, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        base = s.elapsed_time(e) / a.iters
        rec = {"op": name}
        for c in held:
            times = []
            for _ in range(3):
                if c > 0:
                    with torch.cuda.stream(side):
                        ops.cu_hog(sink, c, max(20000.0, base * a.iters * 1e3 * 4))
                    time.sleep(0.002)  # the hog is resident before the timed launches
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times.append(s.elapsed_time(e) / a.iters)
            rec[f"held{c}_ms"] = round(sorted(times)[1], 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
