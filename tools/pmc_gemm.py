"""Tiny driver for PMC passes over one GEMM variant (rocprofv3 --pmc ... -- python tools/pmc_gemm.py <kind> <cfg>).
kind: wgrad_down | wgrad_gateup | dgrad_down | dgrad_down_swiglu | blas_down_dgrad."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
kind, cfg = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0
T = 8192
if kind.startswith("wgrad"):
    N, K = (2048, 11008) if kind == "wgrad_down" else (22016, 2048)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    fn = lambda: ops.wgrad_gemm(out, dy, x, False, cfg)  # noqa: E731
else:
    dy = torch.randn(T, 2048, device="cuda", dtype=torch.bfloat16)
    w = (0.02 * torch.randn(2048, 11008, device="cuda")).to(torch.bfloat16)
    gu = torch.randn(T, 22016, device="cuda", dtype=torch.bfloat16)
    if kind == "dgrad_down":
        fn = lambda: ops.dgrad_gemm(dy, w, None, cfg)  # noqa: E731
    elif kind == "dgrad_down_swiglu":
        fn = lambda: ops.dgrad_gemm(dy, w, gu, cfg)  # noqa: E731
    else:
        fn = lambda: torch.mm(dy, w)  # noqa: E731
for _ in range(5):
    fn()
torch.cuda.synchronize()
