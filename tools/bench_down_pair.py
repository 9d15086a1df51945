"""The down projection's backward pair at M = 8192 (SmolLM3: dy [M, 2048], W_down [2048, 11008], act [M, 11008]):
dgu = swiglu_bwd(dy W, gu) (dgrad with the SwiGLU-backward epilogue: HBM-heavy epilogue) and dW = dy^T act (weight
gradient: compute-heavy), back to back on one stream vs concurrently on two streams (their phases are complementary)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402
from llm_fine_tune_distributed_amd.ops import fused as F  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
M, H, I = 8192, 2048, 11008
dy = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
w = (0.02 * torch.randn(H, I, device="cuda")).to(torch.bfloat16)
gu = torch.randn(M, 2 * I, device="cuda", dtype=torch.bfloat16)
act = torch.randn(M, I, device="cuda", dtype=torch.bfloat16)
dW = torch.zeros(H, I, device="cuda", dtype=torch.bfloat16)
cfg_d = F._dgrad_cfg(dy, swiglu=True)
cfg_w = F._wgrad_cfg(M, H, I)
side = torch.cuda.Stream()
main = torch.cuda.current_stream()


def seq():
    ops.dgrad_gemm(dy, w, gu, cfg_d)
    ops.wgrad_gemm(dW, dy, act, False, cfg_w)


def par():
    side.wait_stream(main)
    with torch.cuda.stream(side):
        ops.wgrad_gemm(dW, dy, act, False, cfg_w)
    ops.dgrad_gemm(dy, w, gu, cfg_d)
    main.wait_stream(side)


def timeit(fn, n=20):
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


res = {"dgrad+swiglu": [], "wgrad": [], "sequential": [], "two streams": []}
for _ in range(3):
    res["dgrad+swiglu"].append(timeit(lambda: ops.dgrad_gemm(dy, w, gu, cfg_d)))
    res["wgrad"].append(timeit(lambda: ops.wgrad_gemm(dW, dy, act, False, cfg_w)))
    res["sequential"].append(timeit(seq))
    res["two streams"].append(timeit(par))
print(f"cfg dgrad {cfg_d} wgrad {cfg_w}")
for k, v in res.items():
    print(f"{k}: {statistics.median(v):.3f} ms")
