"""Model parity vs the installed transformers implementations (CPU, fp32) + structure checks."""
import pytest
import torch

from llm_fine_tune_distributed_amd.models import build_model, smollm3_3b, llama3_8b, tiny, apply_freeze_policy


def _hf(cfg):
    from transformers import LlamaConfig, LlamaForCausalLM, SmolLM3Config, SmolLM3ForCausalLM
    d = cfg.to_hf_dict()
    d.pop("architectures"), d.pop("torch_dtype")
    if cfg.model_type == "smollm3":
        return SmolLM3ForCausalLM(SmolLM3Config(**{k: v for k, v in d.items() if k != "model_type"}))
    d = {k: v for k, v in d.items() if k not in ("model_type", "no_rope_layers", "no_rope_layer_interval")}
    return LlamaForCausalLM(LlamaConfig(**d))


@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_parity_with_transformers(mt):
    torch.manual_seed(0)
    cfg = tiny(mt)
    m = build_model(cfg, dtype=torch.float32)
    hm = _hf(cfg)
    hm.load_state_dict(m.hf_state_dict(), strict=False)
    hm.eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 24))
    labels = ids.clone()
    labels[1, 18:] = -100
    with torch.no_grad():
        ho = hm(input_ids=ids, labels=labels)
        mo = m(ids, labels=labels, return_logits=True)
    assert abs(ho.loss.item() - mo.loss.item()) < 1e-5
    assert (ho.logits.reshape(-1, cfg.vocab_size) - mo.logits).abs().max() < 1e-4


def test_gradients_match_autograd_reference():
    """Fused-op gradients (main_grad path) == plain autograd of the HF model."""
    torch.manual_seed(0)
    cfg = tiny("smollm3")
    m = build_model(cfg, dtype=torch.float32)
    hm = _hf(cfg)
    hm.load_state_dict(m.hf_state_dict(), strict=False)
    for p in m.parameters():
        p.main_grad = torch.zeros_like(p)
    ids = torch.randint(0, cfg.vocab_size, (2, 20))
    m.reset_grad_use_counters()
    m(ids, labels=ids).loss.backward()
    hm(input_ids=ids, labels=ids).loss.backward()
    hsd = dict(hm.named_parameters())
    l0 = m.model.layers[0]
    qkv_ref = torch.cat([hsd[f"model.layers.0.self_attn.{n}_proj.weight"].grad for n in "qkv"], 0)
    assert torch.allclose(l0.self_attn.qkv_proj.main_grad, qkv_ref, atol=1e-5, rtol=1e-3)
    assert torch.allclose(m.model.embed_tokens.main_grad, hsd["model.embed_tokens.weight"].grad, atol=1e-5, rtol=1e-3)
    assert torch.allclose(m.model.norm.weight.main_grad, hsd["model.norm.weight"].grad, atol=1e-5, rtol=1e-3)


def test_packed_equals_padded():
    torch.manual_seed(0)
    cfg = tiny()
    m = build_model(cfg, dtype=torch.float32)
    a = torch.randint(0, cfg.vocab_size, (10,))
    b = torch.randint(0, cfg.vocab_size, (7,))
    # padded batch
    ids = torch.full((2, 10), 2)
    ids[0] = a
    ids[1, :7] = b
    lab = ids.clone()
    lab[1, 7:] = -100
    lp = m(ids, labels=lab).loss
    # packed stream
    ids2 = torch.cat([a, b])
    cu = torch.tensor([0, 10, 17], dtype=torch.int32)
    lab2 = torch.cat([a[1:], torch.tensor([-100]), b[1:], torch.tensor([-100])])
    lk = m(ids2, labels=lab2, cu_seqlens=cu, max_seqlen=10, shift_labels=False).loss
    assert torch.allclose(lp, lk, atol=1e-5)


def test_param_counts_and_freeze_policy():
    c = smollm3_3b()
    assert c.num_parameters() == 3_075_098_624
    assert llama3_8b().num_parameters() == 8_030_261_248
    m = build_model(tiny(), dtype=torch.float32)
    tr, tot = apply_freeze_policy(m, "last_n_layers", n_last=2)
    cfg = m.config
    per_layer = sum(p.numel() for p in m.model.layers[0].parameters())
    assert tr == 2 * per_layer + cfg.vocab_size * cfg.hidden_size  # last 2 layers + tied head
    assert tot == m.num_parameters()


def test_smollm3_nope_layers():
    c = smollm3_3b()
    assert [i for i in range(36) if not c.uses_rope(i)] == list(range(3, 36, 4))


@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_saved_model_loads_in_transformers(tmp_path, mt):
    """save_pretrained() output is a plain HF directory: transformers' AutoModelForCausalLM loads it
    (config.json, safetensors names, tied lm_head dedup) and produces the same logits — the layout that
    downstream tools such as llama.cpp's convert_hf_to_gguf.py read (reference README.md:87-118)."""
    from transformers import AutoModelForCausalLM
    from llm_fine_tune_distributed_amd.train.checkpoint import save_pretrained
    torch.manual_seed(0)
    cfg = tiny(mt)
    m = build_model(cfg, dtype=torch.float32, seed=4)
    save_pretrained(m, str(tmp_path / "out"))
    hm = AutoModelForCausalLM.from_pretrained(str(tmp_path / "out"), torch_dtype=torch.float32)
    hm.eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        ho = hm(input_ids=ids).logits
        mo = m(ids, return_logits=True).logits
    assert (ho.reshape(-1, cfg.vocab_size) - mo).abs().max() < 1e-4


def test_lm_head_loss_gradient_scale():
    """The LM head scales its [T, hidden] operands by the incoming d(loss) (no global unit-gradient switch): the
    trainer's plain loss.backward() and a scaled loss both get the right gradients."""
    import torch
    from llm_fine_tune_distributed_amd import ops
    torch.manual_seed(0)
    h = torch.randn(8, 16, requires_grad=True)
    w = torch.randn(32, 16, requires_grad=True)
    labels = torch.randint(0, 32, (8,))
    inv = torch.tensor([1.0 / 8])

    def grads(scale):
        h.grad = w.grad = None
        loss, _ = ops.lm_head_cross_entropy(h, w, labels, inv)
        (loss if scale is None else loss * scale).backward()
        return h.grad.clone(), w.grad.clone()

    g1, w1 = grads(None)
    gs, ws = grads(1.0)
    g3, w3 = grads(3.0)
    assert torch.equal(g1, gs) and torch.equal(w1, ws)
    assert torch.allclose(g3, 3 * g1, rtol=1e-5) and torch.allclose(w3, 3 * w1, rtol=1e-5)
    hr = h.detach().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    torch.nn.functional.cross_entropy(hr @ wr.t(), labels, reduction="sum").mul(inv[0]).backward()
    assert torch.allclose(g1, hr.grad, atol=1e-5) and torch.allclose(w1, wr.grad, atol=1e-5)
