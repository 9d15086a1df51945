"""Ring-attention building blocks on the HIP kernels (single process): the flash-attention kernel's
per-block output / log-sum-exp, the online merge and the final-lse block backward reproduce full causal
attention for every chunk of a 4-way split. The ring's communication is covered by the gloo tests
(tests/test_context_parallel_cpu.py); this checks what differs on the GPU path."""
import math

import pytest
import torch

from llm_fine_tune_distributed_amd.ops import _ext
from llm_fine_tune_distributed_amd.ops import reference as ref
from llm_fine_tune_distributed_amd.parallel import context_parallel as cp

pytestmark = pytest.mark.gpu


def test_ring_blocks_hip_match_full_attention():
    assert _ext.load(), _ext.load_error()
    torch.manual_seed(0)
    B, L, n, nq, nkv, D = 2, 128, 4, 16, 4, 128
    T = L * n
    qkv = (torch.randn(B * T, (nq + 2 * nkv) * D, device="cuda") * 0.5).to(torch.bfloat16)
    dout = torch.randn(B * T, nq * D, device="cuda").to(torch.bfloat16)
    cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    full = qkv.float().requires_grad_(True)
    o_ref = ref.attention(full, nq, nkv, D, cu, scale, True)
    (g_ref,) = torch.autograd.grad(o_ref, full, dout.float())
    cu_l = torch.arange(0, (B + 1) * L, L, dtype=torch.int32, device="cuda")

    def rows(r):
        return torch.cat([torch.arange(b * T + r * L, b * T + (r + 1) * L, device="cuda") for b in range(B)])

    chunks = [qkv[rows(r)].contiguous() for r in range(n)]
    dkv_tot = [torch.zeros(B * L, 2 * nkv * D, device="cuda") for _ in range(n)]
    for r in range(n):
        q = chunks[r][:, : nq * D]
        o = lse = None
        for src in range(r, -1, -1):  # the ring visits chunks r, r-1, ..., 0 (later ones are skipped)
            o_s, lse_s = cp._block_fwd(q, chunks[src][:, nq * D:], cu_l, L, nq, nkv, D, scale, causal=(src == r))
            o, lse = cp._merge(o, lse, o_s, lse_s, nq, D)
        out = o.to(torch.bfloat16)
        e = (out.float() - o_ref[rows(r)]).norm() / o_ref[rows(r)].norm()
        assert e < 1e-2, (r, e.item())
        dq = torch.zeros(B * L, nq * D, device="cuda")
        for src in range(r, -1, -1):
            dq_s, dkv_s = cp._block_bwd(dout[rows(r)].contiguous(), q, chunks[src][:, nq * D:], out, lse, cu_l, L,
                                        nq, nkv, D, scale, causal=(src == r))
            dq += dq_s
            dkv_tot[src] += dkv_s
        g = g_ref[rows(r)][:, : nq * D]
        assert ((dq - g).norm() / g.norm()).item() < 2e-2, r
    for r in range(n):
        g = g_ref[rows(r)][:, nq * D:]
        assert ((dkv_tot[r] - g).norm() / g.norm()).item() < 2e-2, r
