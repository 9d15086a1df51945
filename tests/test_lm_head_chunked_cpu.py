"""Chunked LM head + CE (ops.fused.LMHeadCEChunkedFn) == the one-pass LMHeadCEFn on CPU (fp32): loss, per-row
stats, dh and dW for chunk sizes that do and do not divide M, through plain autograd, a fresh main_grad (dW written
in the forward, scaled by the upstream gradient in backward) and an accumulating main_grad, plus a whole-model
gradient check with the trainer knob set."""
import pytest
import torch

from llm_fine_tune_distributed_amd import ops
from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.ops.fused import LMHeadCEChunkedFn, LMHeadCEFn


def _data(M=37, K=16, V=50, seed=0):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(M, K, generator=g)
    w = torch.randn(V, K, generator=g) * 0.3
    lab = torch.randint(0, V, (M,), generator=g)
    lab[::5] = -100
    inv = torch.tensor([1.0 / float((lab != -100).sum())])
    return h, w, lab, inv


def _run(fn, h, w, lab, inv, *extra, scale=1.0):
    hh = h.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    loss, stats = fn.apply(hh, ww, lab, inv, *extra)
    (loss * scale).backward()
    return loss.detach(), stats, hh.grad, ww.grad


@pytest.mark.parametrize("chunk", [8, 10, 37, 64])
@pytest.mark.parametrize("scale", [1.0, 2.5])
def test_chunked_matches_one_pass_autograd(chunk, scale):
    h, w, lab, inv = _data()
    l0, s0, dh0, dw0 = _run(LMHeadCEFn, h, w, lab, inv, scale=scale)
    l1, s1, dh1, dw1 = _run(LMHeadCEChunkedFn, h, w, lab, inv, chunk, scale=scale)
    assert torch.allclose(l0, l1, atol=1e-6, rtol=1e-6)
    assert torch.allclose(s0, s1, atol=1e-5, rtol=1e-5)
    assert torch.allclose(dh0, dh1, atol=1e-6, rtol=1e-5)
    assert torch.allclose(dw0, dw1, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("fresh", [True, False])
def test_chunked_main_grad_paths(fresh):
    """fresh: dW goes into main_grad during the forward and is scaled in place by g; not fresh: it is added to the
    previous contents. The ready hook fires once, after the scaling."""
    h, w, lab, inv = _data(M=40)
    _, _, _, dw_ref = _run(LMHeadCEFn, h, w, lab, inv, scale=3.0)
    hh = h.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    prev = torch.randn_like(w)
    ww.main_grad = torch.full_like(w, float("nan")) if fresh else prev.clone()
    ww._sftamd_fresh = fresh
    ww._sftamd_remaining = 1
    fired = []
    ww._sftamd_ready_hook = lambda p: fired.append(p.main_grad.clone())
    loss, _ = LMHeadCEChunkedFn.apply(hh, ww, lab, inv, 16)
    (loss * 3.0).backward()
    want = dw_ref if fresh else prev + dw_ref
    assert ww.grad is None
    assert torch.allclose(ww.main_grad, want, atol=1e-5, rtol=1e-5)
    assert len(fired) == 1 and torch.allclose(fired[0], want, atol=1e-5, rtol=1e-5)
    assert not ww._sftamd_fresh


def test_chunked_no_grad_eval():
    h, w, lab, inv = _data(M=33)
    with torch.no_grad():
        l0, s0 = LMHeadCEFn.apply(h, w, lab, inv)
        l1, s1 = LMHeadCEChunkedFn.apply(h, w, lab, inv, 8)
    assert torch.allclose(l0, l1, atol=1e-6) and torch.allclose(s0, s1, atol=1e-5)


def test_model_gradients_with_chunk_knob():
    """Whole tiny model (tied embedding: the lm_head dW and the embedding backward share main_grad): loss and every
    gradient equal with ops.set_lm_head_chunk on and off."""
    cfg = tiny("smollm3")
    ids = torch.randint(0, cfg.vocab_size, (3, 20), generator=torch.Generator().manual_seed(1))
    labels = ids.clone()
    labels[0, 12:] = -100
    res = {}
    old = ops.lm_head_chunk()
    try:
        for chunk in (0, 16):
            ops.set_lm_head_chunk(chunk)
            m = build_model(cfg, dtype=torch.float32, seed=3)
            for p in m.parameters():
                p.main_grad = torch.zeros_like(p)
            m.reset_grad_use_counters()
            out = m(ids, labels=labels)
            out.loss.backward()
            res[chunk] = (out.loss.detach(), {n: p.main_grad.clone() for n, p in m.named_parameters()})
    finally:
        ops.set_lm_head_chunk(old)
    assert torch.allclose(res[0][0], res[16][0], atol=1e-6)
    for n, g in res[0][1].items():
        assert torch.allclose(g, res[16][1][n], atol=1e-5, rtol=1e-4), n
