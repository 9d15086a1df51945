"""hipBLASLt / rocBLAS forward GEMMs y = x W^T with the WEIGHT's row pitch padded (W a [N, K] view into a [N, K + pad]
buffer): SmolLM3's weights have 4 KiB rows (K = 2048 bf16). TunableOp tunes every (shape, pitch) in this process
(written to gpurun_out/tune_wpitch.csv at exit), then each variant is timed (median of 20), M = 8192.

    python tools/bench_wpitch.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


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


def main():
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    os.makedirs("gpurun_out", exist_ok=True)
    tun.set_filename("gpurun_out/tune_wpitch.csv", insert_device_ordinal=False)
    M = 8192
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(50):
        a @ a
    for name, N, K in (("gate_up", 22016, 2048), ("o_proj", 2048, 2048), ("down", 2048, 11008), ("qkv", 3072, 2048),
                       ("lm_head", 128256, 2048)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        for pad in (0, 64, 128):
            buf = torch.randn(N, K + pad, device="cuda", dtype=torch.bfloat16) * 0.02
            w = buf[:, :K]
            t = timeit(lambda: torch.mm(x, w.t()))
            print(f"{name:8s} W pitch +{pad:3d}: {t:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
