"""Standalone timings of the LoRA streaming kernels (csrc/lora.hip) on the 7B shapes (T = 8192 tokens): lora_fwd (plain
and with the SwiGLU formed on the fly), lora_bwd_dx (plain and writing dgu) and lora_tsum, vs their HBM floor at 8 TB/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def timeit(fn, it=20):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ops = _ext.ops()
    T, H, I, R = 8192, 4096, 11008, 16
    dev = "cuda"
    gu = torch.randn(T, 2 * I, device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, I, device=dev, dtype=torch.bfloat16)
    xh = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    A = torch.randn(R, I, device=dev, dtype=torch.bfloat16) * 0.05
    Ah = torch.randn(3 * R, H, device=dev, dtype=torch.bfloat16) * 0.05
    dxa = torch.randn(T, R, device=dev, dtype=torch.bfloat16)
    dxa2 = torch.randn(T, 2 * R, device=dev, dtype=torch.bfloat16)
    dxah = torch.randn(T, 3 * R, device=dev, dtype=torch.bfloat16)
    base = torch.randn(T, I + 128, device=dev, dtype=torch.bfloat16)[:, :I]
    baseh = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    gb = 1e-9
    rows = [
        ("lora_fwd K=4096 R=48", lambda: ops.lora_fwd(xh, Ah, 0.5, 0.05, 1, H + 128), 2 * T * H * 2),
        ("lora_fwd K=11008 R=16", lambda: ops.lora_fwd(x, A, 0.5, 0.05, 1, I + 128), 2 * T * I * 2),
        ("lora_fwd swiglu K=11008", lambda: ops.lora_fwd(gu, A, 0.5, 0.05, 1, I + 128, False, True), 3 * T * I * 2),
        ("lora_fwd swiglu K=11008 p=0", lambda: ops.lora_fwd(gu, A, 0.5, 0.0, 1, I + 128, False, True), 3 * T * I * 2),
        ("lora_bwd_dx K=4096 R=48", lambda: ops.lora_bwd_dx(baseh, dxah, Ah, 0.05, 1), 2 * T * H * 2),
        ("lora_bwd_dx K=11008 R=16", lambda: ops.lora_bwd_dx(base, dxa, A, 0.05, 1), 2 * T * I * 2),
        ("lora_bwd_dx swiglu K=11008", lambda: ops.lora_bwd_dx(base, dxa, A, 0.05, 1, gu), 5 * T * I * 2),
        ("lora_tsum dA K=4096 R=48", lambda: ops.lora_tsum(xh, H, dxah, 0.05, 1), T * H * 2),
        ("lora_tsum dA K=11008 R=16", lambda: ops.lora_tsum(base, I, dxa, 0.05, 1), T * I * 2),
        ("lora_tsum dA K=11008 p=0", lambda: ops.lora_tsum(base, I, dxa, 0.0, 1), T * I * 2),
        ("lora_tsum dB n=22016 R=32", lambda: ops.lora_tsum(gu, 2 * I, dxa2, 0.0, 0), T * 2 * I * 2),
        ("lora_tsum dB n=4096 R=16", lambda: ops.lora_tsum(xh, H, dxa, 0.0, 0), T * H * 2),
    ]
    # SmolLM3-3B adapter-dx shapes (hidden 2048: qkv R 48, gate_up R 32, o R 16)
    Hs = 2048
    bs = torch.randn(T, Hs + 128, device=dev, dtype=torch.bfloat16)[:, :Hs]
    As = {r: torch.randn(r, Hs, device=dev, dtype=torch.bfloat16) * 0.05 for r in (16, 32, 48)}
    ds = {r: torch.randn(T, r, device=dev, dtype=torch.bfloat16) for r in (16, 32, 48)}
    xs = torch.randn(T, Hs, device=dev, dtype=torch.bfloat16)
    rows += [(f"lora_bwd_dx K=2048 R={r}", lambda r=r: ops.lora_bwd_dx(bs, ds[r], As[r], 0.05, 1), 2 * T * Hs * 2)
             for r in (48, 32, 16)]
    rows += [(f"lora_fwd K=2048 R={r}", lambda r=r: ops.lora_fwd(xs, As[r], 0.5, 0.05, 1, Hs + 128), 2 * T * Hs * 2)
             for r in (48, 32, 16)]
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(200):  # ~1 s of GEMMs first: the clocks ramp up before anything is timed
        a @ a
    for name, fn, nbytes in rows:
        us = timeit(fn)
        print(f"{name:28s} {us:8.1f} us  {nbytes  / (us * 1e-6) * 1e-12:6.2f} TB/s ... floor {nbytes / 8e12 * 1e6:6.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
