"""Tiny driver for PMC passes over the attention kernels (B=16 x T=512, 16q/4kv, d128, causal)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
B, T, NQ, NKV, D = 16, 512, 16, 4, 128
cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device="cuda")
qkv = torch.randn(B * T, (NQ + 2 * NKV) * D, device="cuda", dtype=torch.bfloat16)
dout = torch.randn(B * T, NQ * D, device="cuda", dtype=torch.bfloat16)
ops = _ext.ops()
for _ in range(3):
    out, lse = ops.flash_fwd(qkv, cu, T, NQ, NKV, D, 1 / math.sqrt(D), True)
    ops.flash_bwd(dout, qkv, out, lse, cu, T, NQ, NKV, D, 1 / math.sqrt(D), True)
torch.cuda.synchronize()
