"""Diagnose the interleaved 4-wave ring (wgrad_gemm cfg 14 = reads + DMA interleaved, 15 = reads only, 16 = DMA
only) against cfg 13 and an fp32 reference; localise wrong 32-token steps by masking dy to one step at a time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def rel(a, b):
    return ((a.float() - b).norm() / b.norm()).item()


def main():
    assert _ext.load(), _ext.load_error()
    ops = _ext.ops()
    torch.manual_seed(0)
    T, N, K = 1024, 768, 1024
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    for cfg in (13, 14, 15, 16):
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        ops.wgrad_gemm(out, dy, x, False, cfg)
        torch.cuda.synchronize()
        e = rel(out, ref)
        print(f"wgrad cfg {cfg}: rel err {e:.2e}", flush=True)
        if e > 5e-3:
            bad = []
            for s in range(T // 32):
                d1 = torch.zeros_like(dy)
                d1[32 * s:32 * s + 32] = dy[32 * s:32 * s + 32]
                ops.wgrad_gemm(out, d1, x, False, cfg)
                r1 = d1.float().t() @ x.float()
                if rel(out, r1) > 5e-3:
                    bad.append((s, round(rel(out, r1), 3)))
            print(f"  wrong steps: {bad}", flush=True)
            diff = (out.float() - ref).abs().reshape(N // 128, 128, K // 128, 128).amax(dim=(1, 3))
            print("  max err per 128x128 wave tile (rows = N/128):")
            print(diff.cpu().numpy().round(1), flush=True)
    M, Kd, Nd = 1024, 4608, 768
    dyd = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
    w = (0.02 * torch.randn(Kd, Nd, device="cuda")).to(torch.bfloat16)
    refd = dyd.float() @ w.float()
    for cfg in (13, 14):
        o = ops.dgrad_gemm(dyd, w, None, cfg)
        torch.cuda.synchronize()
        print(f"dgrad cfg {cfg}: rel err {rel(o, refd):.2e}", flush=True)


if __name__ == "__main__":
    main()
