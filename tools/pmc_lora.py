"""Tiny driver for PMC passes over the LoRA streaming kernels at the SmolLM3-3B MLP shapes (T = 8192): lora_fwd with
the SwiGLU formed on the fly (R = 16, K = 11008), lora_fwd at K = 2048 / R = 48 (qkv), lora_bwd_dx writing dgu, and
the plain SwiGLU kernel as a streaming reference, and the adapter-gradient reductions (down dA, gate_up dB^T)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
T, H, I, R = 8192, 2048, 11008, 16
gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
xh = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
A = torch.randn(R, I, device="cuda", dtype=torch.bfloat16) * 0.05
Ah = torch.randn(3 * R, H, device="cuda", dtype=torch.bfloat16) * 0.05
dxa = torch.randn(T, R, device="cuda", dtype=torch.bfloat16)
dxa2 = torch.randn(T, 2 * R, device="cuda", dtype=torch.bfloat16)
base = torch.randn(T, I + 128, device="cuda", dtype=torch.bfloat16)[:, :I]
for _ in range(3):
    ops.lora_fwd(gu, A, 0.5, 0.05, 1, I + 128, False, True)
    ops.lora_fwd(xh, Ah, 0.5, 0.05, 1, H + 128)
    ops.lora_bwd_dx(base, dxa, A, 0.05, 1, gu)
    ops.swiglu_fwd(gu)
    Xw = ops.lora_fwd(gu, A, 0.5, 0.05, 1, I + 128, False, True)[0]
    ops.lora_tsum(Xw, I, dxa, 0.05, 1)                    # dA of the down projection (256-column workgroups)
    ops.lora_tsum(gu, 2 * I, dxa2, 0.0, 0)                 # dB^T of gate_up
torch.cuda.synchronize()
