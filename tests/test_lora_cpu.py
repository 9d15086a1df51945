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


def _unfused_with_dropout(x, w, lora):
    """Reference LoRA math with the framework's hash dropout (same seed draw as ops.lora_linear)."""
    import llm_fine_tune_distributed_amd.ops as ops
    p = lora.dropout.p if lora.training else 0.0
    seed = int(torch.randint(1, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
    x2d = x.reshape(-1, x.shape[-1])
    xd = ops.reference.dropout_add(None, x2d, p, seed) if p > 0 else x2d
    outs = [xd @ a.t() @ b.t() if act else x2d.new_zeros(x2d.shape[0], n)
            for a, b, n, act in zip(lora.A, lora.B, lora.out_splits, lora.active)]
    y = x2d @ w.t() + torch.cat(outs, -1) * lora.scaling
    return y.view(*x.shape[:-1], -1)


def test_lora_wide_with_dropout_matches_reference():
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32)
    apply_lora(m, LoRAConfig(r=4, lora_alpha=8, lora_dropout=0.2))
    for l in m.model.layers:
        for fl in (l.self_attn.lora["qkv"], l.mlp.lora["gate_up"], l.mlp.lora["down"]):
            for b in fl.B:
                torch.nn.init.normal_(b, std=0.1)
    m.train()
    ids = torch.randint(0, 1000, (2, 12))
    torch.manual_seed(123)
    out = m(ids, labels=ids)
    out.loss.backward()
    g1 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    import llm_fine_tune_distributed_amd.models.transformer as T
    orig = T.ops.lora_linear
    T.ops.lora_linear = _unfused_with_dropout
    try:
        for p in m.parameters():
            p.grad = None
        torch.manual_seed(123)
        out2 = m(ids, labels=ids)
        out2.loss.backward()
    finally:
        T.ops.lora_linear = orig
    assert torch.allclose(out.loss, out2.loss, atol=1e-5), (out.loss, out2.loss)
    for n, p in m.named_parameters():
        if p.grad is not None:
            assert torch.allclose(g1[n], p.grad, atol=1e-5, rtol=1e-3), n


def test_hash_dropout_statistics():
    from llm_fine_tune_distributed_amd.ops import reference as ref
    b = torch.ones(256, 512)
    y = ref.dropout_add(None, b, 0.25, 7)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.75) < 0.01
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1 / 0.75))
    y2 = ref.dropout_add(b, b, 0.25, 7)
    assert torch.allclose(y2, y + 1)
    assert not torch.equal(ref.dropout_add(None, b, 0.25, 8), y)


def test_save_merged_lora_loads_in_transformers(tmp_path):
    """save_pretrained(merge_lora=True): adapters folded into copies of the base weights (the live model
    keeps its adapters); transformers loads the directory and reproduces the adapted model's logits."""
    import os
    from transformers import AutoModelForCausalLM
    from llm_fine_tune_distributed_amd.train.checkpoint import save_pretrained
    torch.manual_seed(0)
    m = build_model(tiny("smollm3"), dtype=torch.float32, seed=5)
    apply_lora(m, LoRAConfig(r=4, lora_alpha=8, lora_dropout=0.0, target_modules=["q_proj", "v_proj", "o_proj",
                                                                                   "up_proj", "down_proj"]))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if ".lora." in n and p.numel() > 0:
                p.normal_(0.0, 0.05)
    m.eval()
    ids = torch.randint(0, m.config.vocab_size, (2, 16))
    with torch.no_grad():
        mo = m(ids, return_logits=True).logits
    save_pretrained(m, str(tmp_path / "merged"), merge_lora=True)
    save_pretrained(m, str(tmp_path / "adapters"))
    assert not os.path.exists(tmp_path / "merged" / "adapter_model.safetensors")
    assert os.path.exists(tmp_path / "adapters" / "adapter_model.safetensors")
    assert m.model.layers[0].self_attn.lora is not None  # live model untouched
    hm = AutoModelForCausalLM.from_pretrained(str(tmp_path / "merged"), torch_dtype=torch.float32).eval()
    with torch.no_grad():
        ho = hm(input_ids=ids).logits
    assert (ho.reshape(mo.shape) - mo).abs().max() < 1e-4
    base = AutoModelForCausalLM.from_pretrained(str(tmp_path / "adapters"), torch_dtype=torch.float32).eval()
    with torch.no_grad():
        bo = base(input_ids=ids).logits
    assert (bo.reshape(mo.shape) - mo).abs().max() > 1e-3  # base weights alone differ: the merge did something


def test_wide_weight_follows_adapter_updates():
    """The B blocks of the wide weight are re-copied only when an adapter changed (version counters): a forward
    after an in-place update (what the optimizer does through the flat buffer) uses the new B; a repeated
    forward with unchanged adapters copies nothing."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32)
    apply_lora(m, LoRAConfig(r=4, lora_alpha=8, lora_dropout=0.0))
    fl = m.model.layers[0].mlp.lora["gate_up"]
    K = fl.in_features
    ids = torch.randint(0, 1000, (2, 12))
    m(ids, labels=ids)
    key = fl.wide._sftamd_bkey
    m(ids, labels=ids)
    assert fl.wide._sftamd_bkey == key  # nothing changed: no copy
    with torch.no_grad():
        fl.B[1].add_(0.5)  # bumps the version counter like the optimizer's increment_version
    m(ids, labels=ids)
    assert fl.wide._sftamd_bkey != key
    o, rows, c = fl.wide_meta[1]
    assert torch.equal(fl.wide[o:o + rows, K + c:K + c + fl.r], fl.B[1].detach())
    assert F._sync_wide is not None


def test_lora_trainer_updates_reach_the_wide_weight(tmp_path):
    """Through the real engine (adapters relocated into the flat parameter buffer) and the optimizer (a raw in-place
    update + increment_version): after a training step the wide weight's B blocks equal the updated adapters."""
    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32)
    ds = TokenizedDataset.synthetic(16, m.config.vocab_size, 6, 12, seed=3)
    a = SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=4, max_steps=2, learning_rate=1e-2,
                  jsonl_log=False, logging_steps=0, save_strategy="no", freeze_policy="lora", lora_dropout=0.0)
    t = SFTTrainer(model=m, args=a, train_dataset=ds)
    t.train()
    fl = m.model.layers[1].self_attn.lora["qkv"]
    ids = torch.randint(0, 1000, (2, 12))
    m(ids, labels=ids)  # the next forward syncs the last update
    K = fl.in_features
    for (o, rows, c), B in zip(fl.wide_meta, fl.B):
        assert B.detach().abs().sum() > 0  # trained away from the zero init
        assert torch.equal(fl.wide[o:o + rows, K + c:K + c + fl.r], B.detach())


def test_prewidened_view_detection(monkeypatch):
    """_prewidened (the in-place LoRA widening): only a norm output add_rms_norm marked as the left [T, K] block of its
    own [T, ldX] buffer (``_sftamd_wide_ld``), at a shape the widening kernel takes (K % 256, R a multiple of 16 in
    16..64), is taken as X'. An unmarked view with the same strides (e.g. a column slice of someone else's
    activation), an unsupported rank (qkv r = 8: R = 24; r = 32: R = 96), other widths, short storages and non-bf16
    inputs are not."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    monkeypatch.setattr(F._ext, "use_hip", lambda t: True)
    T, K, ldX = 6, 256, 384
    acat = torch.zeros(48, K, dtype=torch.bfloat16)
    buf = torch.zeros(T, ldX, dtype=torch.bfloat16)
    x = buf[:, :K]
    assert F._prewidened(x, x, ldX, acat) is None  # not marked by the norm
    x._sftamd_wide_ld = ldX
    X = F._prewidened(x, x, ldX, acat)
    assert X is not None and X.shape == (T, ldX) and X.data_ptr() == buf.data_ptr() and X.stride() == (ldX, 1)
    X[:, K:] = 1  # the view covers the buffer's adapter / padding columns
    assert (buf[:, K:] == 1).all()
    for R in (24, 96, 8):
        assert F._prewidened(x, x, ldX, torch.zeros(R, K, dtype=torch.bfloat16)) is None, R
    assert F._prewidened(x, x, ldX + 8, acat) is None                                    # another width
    c = torch.zeros(T, K, dtype=torch.bfloat16)
    c._sftamd_wide_ld = ldX
    assert F._prewidened(c, c, ldX, acat) is None                                        # contiguous [T, K]
    short = torch.zeros(T * ldX - 8, dtype=torch.bfloat16).as_strided((T, K), (ldX, 1))
    short._sftamd_wide_ld = ldX
    assert F._prewidened(short, short, ldX, acat) is None                                # rows past the storage
    xf = buf[:, :K].float()
    xf._sftamd_wide_ld = ldX
    assert F._prewidened(xf, xf, ldX, acat) is None                                      # not bf16


def test_wide_ld_only_for_supported_ranks():
    """The norm writes into the consumer's widened buffer only where the widening kernel takes the shape: qkv with
    r = 8 (R = 24) or r = 32 (R = 96) gets a plain y (the copying widening runs instead of failing)."""
    import llm_fine_tune_distributed_amd.models.transformer as TR
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.models.lora import LoRAConfig, apply_lora
    for r, want in ((16, True), (8, False), (32, False)):
        cfg = tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=1, head_dim=128, intermediate_size=512,
                   vocab_size=512, num_hidden_layers=1)
        m = build_model(cfg, dtype=torch.float32, seed=0)
        apply_lora(m, LoRAConfig(r=r, lora_alpha=8))
        at = m.model.layers[0].self_attn
        fl = at.lora["qkv"]
        if getattr(fl, "wide", None) is None:
            continue  # no wide weight on this path: nothing is widened in place
        assert (TR._wide_ld(at.lora, "qkv", at.qkv_proj) > 0) == want, r
