"""Is the 4-wave kernel's input-gradient form slower because of its ROW operand? The SmolLM3 gate_up input gradient
dX[8192, 2048] = dgu[8192, 22016] . W[22016, 2048] runs at ~1.37 PF/s in the step, the weight gradients of the same
FLOPs at ~1.7. This times the same product (M = 8192, N = 2048, reduction 22016, 256 tiles = one round) in both
layouts the kernel has:

  ROW / TR  (dgrad_gemm cfg 12 / 13):  A = dgu [8192, 22016] row-major (reduction contiguous), B = W [22016, 2048]
  TR  / TR  (wgrad_gemm cfg 12 / 13):  A = dgu^T [22016, 8192] (reduction is the row index), B = W

and the down weight gradient shape (TR / TR, reduction 8192, 344 tiles) for reference. Median of 20, us.

    python tools/bench_g4_layout.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


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
    return statistics.median(ts) * 1e3


def fb(on):  # temporary A/B switch of the read schedule (csrc/gemm_4w.hip)
    os.environ["SFTAMD_G4_FB"] = "1" if on else "0"


def main():
    assert _ext.load(), _ext.load_error()
    ops = _ext.ops()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(100):
        a @ a
    del a
    M, N, R = 8192, 2048, 22016
    dy = torch.randn(M, R, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(R, N, device="cuda", dtype=torch.bfloat16) * 0.02
    dyt = dy.t().contiguous()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * R
    ref = ops.dgrad_gemm(dy, w, None, 13)
    for cfg in (12, 13):
        ops.wgrad_gemm(out, dyt, w, False, cfg)
        err = (out.float() - ref.float()).abs().max().item()
        print(f"TR/TR cfg {cfg} vs ROW/TR cfg 13 max |diff| {err:.3e}", flush=True)
    for on in (0, 1):
        fb(on)
        for cfg in (12, 13):
            o2 = ops.dgrad_gemm(dy, w, None, cfg)
            ops.wgrad_gemm(out, dyt, w, False, cfg)
            print(f"FB={on} cfg {cfg}: dgrad |diff| {(o2.float() - ref.float()).abs().max().item():.3e} "
                  f"wgrad-form |diff| {(out.float() - ref.float()).abs().max().item():.3e}", flush=True)
    for rep in range(2):
        for on in (0, 1):
            fb(on)
            for cfg in (12, 13):
                t = timeit(lambda: ops.dgrad_gemm(dy, w, None, cfg))
                print(f"FB={on} ROW/TR dgrad cfg {cfg}: {t:8.1f} us  {fl / t / 1e9:6.3f} PF/s", flush=True)
                t = timeit(lambda: ops.wgrad_gemm(out, dyt, w, False, cfg))
                print(f"FB={on} TR/TR  wgrad cfg {cfg}: {t:8.1f} us  {fl / t / 1e9:6.3f} PF/s", flush=True)
    # down weight gradient: dW[2048, 11008] = dy[8192, 2048]^T act[8192, 11008]
    dyd = torch.randn(8192, 2048, device="cuda", dtype=torch.bfloat16)
    act = torch.randn(8192, 11008, device="cuda", dtype=torch.bfloat16)
    dw = torch.empty(2048, 11008, device="cuda", dtype=torch.bfloat16)
    fl2 = 2.0 * 8192 * 2048 * 11008
    x = torch.randn(8192, 2048, device="cuda", dtype=torch.bfloat16)
    dwg = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
    # small shapes of the step: o_proj / qkv input gradients (K = 2048 / 3072, cfg 12), qkv weight gradient (1212)
    dyo = torch.randn(8192, 2048, device="cuda", dtype=torch.bfloat16)
    wo = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    dyq = torch.randn(8192, 3072, device="cuda", dtype=torch.bfloat16)
    wq = torch.randn(3072, 2048, device="cuda", dtype=torch.bfloat16)
    dwq = torch.empty(3072, 2048, device="cuda", dtype=torch.bfloat16)
    for rep in range(2):
        for on in (0, 1):
            fb(on)
            for cfg in (13, 1213):
                t = timeit(lambda: ops.wgrad_gemm(dw, dyd, act, False, cfg))
                print(f"FB={on} down wgrad cfg {cfg}: {t:8.1f} us  {fl2 / t / 1e9:6.3f} PF/s", flush=True)
            # gate_up weight gradient: dW[22016, 2048] = dgu[8192, 22016]^T x[8192, 2048] (688 tiles)
            t = timeit(lambda: ops.wgrad_gemm(dwg, dy, x, False, 13))
            print(f"FB={on} gate_up wgrad cfg 13: {t:8.1f} us  {fl / t / 1e9:6.3f} PF/s", flush=True)
            t = timeit(lambda: ops.dgrad_gemm(dyo, wo, None, 12))
            print(f"FB={on} o dgrad cfg 12: {t:8.1f} us", flush=True)
            t = timeit(lambda: ops.dgrad_gemm(dyq, wq, None, 12))
            print(f"FB={on} qkv dgrad cfg 12: {t:8.1f} us", flush=True)
            t = timeit(lambda: ops.wgrad_gemm(dwq, dyq, x, False, 1212))
            print(f"FB={on} qkv wgrad cfg 1212: {t:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
