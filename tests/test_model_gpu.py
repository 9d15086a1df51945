"""Whole-model numerics on GPU: HIP kernel path vs the PyTorch reference path (same weights)."""
import os

import pytest
import torch

from llm_fine_tune_distributed_amd.models import build_model, tiny

pytestmark = pytest.mark.gpu


def _run(model, ids, labels, hip: bool):
    os.environ["SFTAMD_DISABLE_HIP"] = "0" if hip else "1"
    try:
        for p in model.parameters():
            p.grad = None
        model.reset_grad_use_counters()
        out = model(ids, labels=labels)
        out.loss.backward()
        grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}
        return out.loss.detach().float(), grads
    finally:
        os.environ["SFTAMD_DISABLE_HIP"] = "0"


@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_model_hip_vs_reference(mt):
    torch.manual_seed(0)
    cfg = tiny(mt, hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
               intermediate_size=1024, vocab_size=1024, num_hidden_layers=4)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    ids = torch.randint(0, 1024, (4, 200), device="cuda")
    labels = ids.clone()
    labels[:, 150:] = -100
    l_hip, g_hip = _run(m, ids, labels, True)
    l_ref, g_ref = _run(m, ids, labels, False)
    assert abs(l_hip.item() - l_ref.item()) < 2e-2 * abs(l_ref.item())
    for n in g_ref:
        e = (g_hip[n] - g_ref[n]).norm() / (g_ref[n].norm() + 1e-12)
        assert e < 5e-2, (n, e.item())
