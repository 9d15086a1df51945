"""LoRA fused linear == unfused reference (outputs and adapter/input gradients)."""
import torch

from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.models.lora import LoRAConfig, apply_lora


def test_lora_linear_matches_module_math():
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32)
    apply_lora(m, LoRAConfig(r=4, lora_alpha=8, lora_dropout=0.0))
    for l in m.model.layers:
        for fl in (l.self_attn.lora["qkv"], l.mlp.lora["gate_up"]):
            for b in fl.B:
                torch.nn.init.normal_(b, std=0.1)
    ids = torch.randint(0, 1000, (2, 12))
    out = m(ids, labels=ids)
    out.loss.backward()
    g_fused = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    # unfused reference: the FusedLoRA module's own forward (cat of per-adapter products)
    import llm_fine_tune_distributed_amd.ops as ops
    import llm_fine_tune_distributed_amd.models.transformer as T
    orig = ops.lora_linear

    def unfused(x, w, lora):
        return ops.linear(x, w) + lora(x)
    T.ops.lora_linear = unfused
    try:
        for p in m.parameters():
            p.grad = None
        out2 = m(ids, labels=ids)
        out2.loss.backward()
    finally:
        T.ops.lora_linear = orig
    assert torch.allclose(out.loss, out2.loss, atol=1e-6)
    for n, p in m.named_parameters():
        if p.grad is not None:
            assert torch.allclose(g_fused[n], p.grad, atol=1e-6, rtol=1e-4), n
