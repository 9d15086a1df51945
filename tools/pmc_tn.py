"""One forward-layout GEMM variant for PMC passes: rocprofv3 --pmc ... -- python tools/pmc_tn.py <cfg|blas> [N K]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
cfg = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 22016
K = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
x = torch.randn(8192, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
fn = (lambda: torch.nn.functional.linear(x, w)) if cfg == "blas" else (lambda: ops.gemm_tn(x, w, int(cfg)))
for _ in range(5):
    fn()
torch.cuda.synchronize()
