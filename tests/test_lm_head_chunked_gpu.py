"""Chunked LM head + CE on the GPU at the SmolLM3 vocabulary (128256 x 2048, bf16): loss, dh and dW (fresh
main_grad, written by the ring wgrad kernel chunk by chunk) vs the one-pass path and the fp32 reference, and the
peak-memory saving (the [M, V] logits never exist)."""
import pytest
import torch

from llm_fine_tune_distributed_amd.ops import _ext
from llm_fine_tune_distributed_amd.ops.fused import LMHeadCEChunkedFn, LMHeadCEFn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _case(fn, h, w, lab, inv, *extra):
    hh = h.clone().requires_grad_(True)
    ww = w.clone()
    ww.requires_grad_(True)
    ww.main_grad = torch.empty_like(w)
    ww._sftamd_fresh = True
    ww._sftamd_remaining = 1
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    loss, _ = fn.apply(hh, ww, lab, inv, *extra)
    loss.backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    return loss.detach().float(), hh.grad, ww.main_grad, peak


def test_chunked_lm_head_smollm3_vocab():
    assert _ext.load(), _ext.load_error()
    torch.manual_seed(0)
    M, K, V = 4096, 2048, 128256
    h = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (0.02 * torch.randn(V, K, device="cuda")).to(torch.bfloat16)
    lab = torch.randint(0, V, (M,), device="cuda")
    lab[::7] = -100
    inv = (1.0 / (lab != -100).sum().float()).reshape(1)
    l0, dh0, dw0, peak0 = _case(LMHeadCEFn, h, w, lab, inv)
    l1, dh1, dw1, peak1 = _case(LMHeadCEChunkedFn, h, w, lab, inv, 1024)
    # fp32 reference
    hf = h.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    logits = hf @ wf.t()
    lr = torch.nn.functional.cross_entropy(logits, lab, ignore_index=-100, reduction="sum") * inv[0]
    lr.backward()
    assert abs(l1.item() - lr.item()) < 1e-2 * abs(lr.item())
    assert abs(l1.item() - l0.item()) < 1e-3 * abs(l0.item())
    assert _rel(dh1, hf.grad) < 2e-2 and _rel(dh1, dh0) < 1e-2
    assert _rel(dw1, wf.grad) < 2e-2 and _rel(dw1, dw0) < 1e-2
    # one-pass peak holds the [M, V] bf16 logits (1.05 GB here); chunked holds a [1024, V] chunk (0.26 GB)
    assert peak0 - peak1 > 0.6e9, (peak0, peak1)
