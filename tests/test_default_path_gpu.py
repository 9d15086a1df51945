"""The SHIPPED default path at real SmolLM3-3B widths (hidden 2048, 16 q / 4 kv heads x 128, intermediate 11008),
4 layers (one NoPE), reduced vocabulary, 16 x 512 tokens: every dispatch decision runs with NO environment override
(tests/test_env_guard.py), and the kernel variants that actually launched are read back from the native dispatch
trace (csrc/dispatch_trace.cpp). Loss, every parameter gradient (read from the DDP engine's flat buffer, where the
fused ops write them) and the clip norm from the fused wgrad-epilogue norm slots are compared against the fp32
PyTorch reference model with the same weights."""
import pytest
import torch

from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _trace():
    out = {}
    for item in _ext.ops().dispatch_trace_read().split(";"):
        if item:
            k, v = item.split("=")
            out[k] = int(v)
    return out


def _cfg():
    return tiny("smollm3", hidden_size=2048, num_attention_heads=16, num_key_value_heads=4, head_dim=128,
                intermediate_size=11008, vocab_size=8192, num_hidden_layers=4, max_position_embeddings=4096,
                rope_theta=2e6)


def test_default_path_smollm3_widths_vs_fp32_reference(monkeypatch):
    from llm_fine_tune_distributed_amd.parallel.ddp import DDPEngine
    assert _ext.load(), _ext.load_error()
    torch.manual_seed(0)
    cfg = _cfg()
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=11)
    ref = build_model(cfg, device="cuda", dtype=torch.float32, seed=11)
    with torch.no_grad():
        for (n, p), (n2, q) in zip(m.named_parameters(), ref.named_parameters()):
            assert n == n2
            q.copy_(p.float())
    B, T = 16, 512
    ids = torch.randint(0, cfg.vocab_size, (B, T), device="cuda")
    labels = ids.clone()
    labels[:, 400:] = -100  # padded-batch style ignored tail

    eng = DDPEngine(m, 1, 0)  # world 1 on GPU: gradients into the flat buffer, fused clip-norm slots
    assert eng.fused_norm
    m.train()
    _ext.ops().dispatch_trace(True)
    try:
        eng.zero_grad()
        eng.prepare_backward()
        out = m(ids, labels=labels)
        out.loss.backward()
        eng.finish_backward()
        norm2 = eng.grad_norm_sq()
        torch.cuda.synchronize()
    finally:
        _ext.ops().dispatch_trace(False)
    tr = _trace()
    # ---- which variants ran (the defaults of ops/fused.py and the C++ launchers at these shapes)
    assert tr.get("tn.rope.c11", 0) == 3 and tr.get("tn.rope.tail", 0) == 3, tr  # qkv + RoPE, 384-tile tail split
    assert tr.get("attn.fwd32", 0) == 4 and tr.get("attn.dkdv32", 0) == 4 and tr.get("attn.dq32", 0) == 4, tr
    assert tr.get("attn.bwd_rope_epi", 0) == 3, tr  # inverse RoPE in the dq / dK epilogues of the 3 RoPE layers
    # wgrad: the 4-wave ring (csrc/gemm_4w.hip) for gate_up and, hybrid split-K, down_proj; the 4-wave kernel split 2
    # ways over the tokens for qkv; 8-wave rings for lm_head (8192-vocab: 256 tiles of 256 x 128) / o_proj (split 2)
    for c in (13, 1213, 9, 209, 1212):
        assert tr.get(f"wgrad.c{c}", 0) > 0, (c, tr)
    assert tr.get("wgrad.norm_slots", 0) > 0, tr
    assert tr.get("dgrad.swiglu.c7", 0) >= 4 and tr.get("dgrad.tail", 0) > 0, tr  # down dgrad + SwiGLU bwd
    assert tr.get("dgrad.c12", 0) > 0, tr  # o_proj / qkv dgrads: 4-wave pair loop
    assert tr.get("dgrad.c13", 0) >= 5, tr  # gate_up (K = 22016) x 4 + lm_head: 4-wave ring
    assert "attn.dq3" not in tr, tr  # (the recompute path: past the dS^T budget only)
    # ---- numerics vs the fp32 reference path (same weights, PyTorch ops)
    monkeypatch.setenv("SFTAMD_DISABLE_HIP", "1")
    ref.train()
    out_r = ref(ids, labels=labels)
    out_r.loss.backward()
    monkeypatch.delenv("SFTAMD_DISABLE_HIP")
    assert abs(out.loss.item() - out_r.loss.item()) < 2e-2 * abs(out_r.loss.item())
    gref = {n: p.grad.float() for n, p in ref.named_parameters()}
    total_ref = 0.0
    for p, _, _, _ in eng.layout:
        name = eng.param_names[id(p)]
        g = p.main_grad.float()
        e = ((g - gref[name]).norm() / (gref[name].norm() + 1e-12)).item()
        assert e < 5e-2, (name, e)
        total_ref += gref[name].pow(2).sum().item()
    # the clip norm from the wgrad-epilogue slots + the leftover pass == the reference gradient norm
    assert norm2 is not None
    assert abs(norm2.sqrt().item() - total_ref ** 0.5) < 3e-2 * total_ref ** 0.5
