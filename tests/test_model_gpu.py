"""Whole-model numerics on GPU: HIP kernel path vs the PyTorch reference path (same weights)."""
import os

import pytest
import torch

from llm_fine_tune_distributed_amd.models import build_model, tiny

pytestmark = pytest.mark.gpu


def _run(model, ids, labels, hip: bool):
    prev = os.environ.get("SFTAMD_DISABLE_HIP")
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
        if prev is None:
            os.environ.pop("SFTAMD_DISABLE_HIP", None)
        else:
            os.environ["SFTAMD_DISABLE_HIP"] = prev


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


@pytest.mark.parametrize("down_fused", [True, False])
@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_model_fused_gemm_epilogues(mt, down_fused, monkeypatch):
    """M = 1024 tokens (multiple of 256): qkv+RoPE and gate_up+SwiGLU run as single HIP GEMMs with fused
    epilogues (csrc/gemm_tn.hip); loss and every gradient match the unfused HIP path (hipBLASLt + kernels)
    and the PyTorch reference."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    torch.manual_seed(0)
    cfg = tiny(mt, hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
               intermediate_size=1024, vocab_size=1024, num_hidden_layers=4)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    ids = torch.randint(0, 1024, (4, 256), device="cuda")
    labels = ids.clone()
    labels[:, 200:] = -100
    calls = {"swiglu": 0, "rope": 0}
    # down_fused: gate_up GEMM + SwiGLU epilogue feeding the down GEMM whose dgrad carries the SwiGLU backward
    # (GateUpActFn + SwiGLUDownFn); else GateUpSwiGLUFn + a plain down projection
    sw_fn = F.GateUpActFn if down_fused else F.GateUpSwiGLUFn
    monkeypatch.setattr(F, "_SWIGLU_DOWN", down_fused)
    orig_sw, orig_rope, orig_ra = sw_fn.apply, F.QKVRopeFn.apply, F.QKVRopeAttnFn.apply

    def sw(*a):
        calls["swiglu"] += 1
        return orig_sw(*a)

    def rp(*a):
        calls["rope"] += 1
        return orig_rope(*a)

    def ra(*a):  # qkv + RoPE GEMM fused with the attention node (default for RoPE layers)
        calls["rope"] += 1
        return orig_ra(*a)

    monkeypatch.setattr(sw_fn, "apply", sw)
    monkeypatch.setattr(F.QKVRopeFn, "apply", rp)
    monkeypatch.setattr(F.QKVRopeAttnFn, "apply", ra)
    monkeypatch.setattr(F, "_TN_MODE", "1")
    l_f, g_f = _run(m, ids, labels, True)
    assert calls["swiglu"] == 4 and calls["rope"] == (3 if mt == "smollm3" else 4)  # NoPE layer 3
    monkeypatch.setattr(F, "_TN_MODE", "0")
    l_u, g_u = _run(m, ids, labels, True)
    l_r, g_r = _run(m, ids, labels, False)
    assert abs(l_f.item() - l_u.item()) < 5e-3 * abs(l_u.item())
    assert abs(l_f.item() - l_r.item()) < 2e-2 * abs(l_r.item())
    for n in g_u:
        e = (g_f[n] - g_u[n]).norm() / (g_u[n].norm() + 1e-12)
        assert e < 2e-2, (n, e.item())
        e = (g_f[n] - g_r[n]).norm() / (g_r[n].norm() + 1e-12)
        assert e < 5e-2, (n, e.item())


@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_model_rope_attention_node(mt, monkeypatch):
    """qkv GEMM (+RoPE epilogue) + flash attention as ONE autograd node whose backward inverts the RoPE inside the
    attention kernels' dq / dK epilogues == the two separate nodes (rope kernel on dqkv), and == the reference."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    torch.manual_seed(0)
    cfg = tiny(mt, hidden_size=512, num_attention_heads=8, num_key_value_heads=2, head_dim=128,
               intermediate_size=1024, vocab_size=1024, num_hidden_layers=4)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    ids = torch.randint(0, 1024, (4, 256), device="cuda")
    labels = ids.clone()
    labels[:, 200:] = -100
    n = {"fused": 0}
    orig = F.QKVRopeAttnFn.apply

    def ra(*a):
        n["fused"] += 1
        return orig(*a)

    monkeypatch.setattr(F.QKVRopeAttnFn, "apply", ra)
    monkeypatch.setattr(F, "_ROPE_ATTN_FUSED", True)
    l_f, g_f = _run(m, ids, labels, True)
    assert n["fused"] == (3 if mt == "smollm3" else 4)  # NoPE layer 3 keeps the plain projection
    monkeypatch.setattr(F, "_ROPE_ATTN_FUSED", False)
    l_s, g_s = _run(m, ids, labels, True)
    assert n["fused"] == (3 if mt == "smollm3" else 4)
    l_r, g_r = _run(m, ids, labels, False)
    assert torch.equal(l_f, l_s)  # same forward kernels
    for k in g_s:
        e = (g_f[k] - g_s[k]).norm() / (g_s[k].norm() + 1e-12)
        assert e < 1e-2, (k, e.item())
        e = (g_f[k] - g_r[k]).norm() / (g_r[k].norm() + 1e-12)
        assert e < 5e-2, (k, e.item())


@pytest.mark.parametrize("mt", ["smollm3", "llama"])
def test_model_attention_delta_handoff(mt, monkeypatch):
    """o_proj's backward computing the attention backward's delta in its dgrad epilogue (AttnOutLinearFn, handed to
    QKVRopeAttnFn / FlashAttnFn through the layer's box) == the attention node's own delta kernel, on RoPE and NoPE
    layers, and == the fp32 reference."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    torch.manual_seed(0)
    cfg = tiny(mt, hidden_size=512, num_attention_heads=8, num_key_value_heads=2, head_dim=128,
               intermediate_size=1024, vocab_size=1024, num_hidden_layers=4)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    ids = torch.randint(0, 1024, (4, 256), device="cuda")
    labels = ids.clone()
    labels[:, 200:] = -100
    n = {"delta": 0, "used": 0}
    orig_op, orig_take = F.AttnOutLinearFn.apply, F._take_delta

    def op(*a):
        n["delta"] += 1
        return orig_op(*a)

    def take(*a):
        d = orig_take(*a)
        n["used"] += d is not None
        return d

    monkeypatch.setattr(F.AttnOutLinearFn, "apply", op)
    monkeypatch.setattr(F, "_take_delta", take)
    monkeypatch.setattr(F, "_DELTA_FUSED", True)
    l_f, g_f = _run(m, ids, labels, True)
    assert n["delta"] == 4 and n["used"] == 4, n  # every layer, NoPE layer 3 included
    monkeypatch.setattr(F, "_DELTA_FUSED", False)
    l_s, g_s = _run(m, ids, labels, True)
    assert n["delta"] == 4 and n["used"] == 4, n
    l_r, g_r = _run(m, ids, labels, False)
    assert torch.equal(l_f, l_s)  # same forward kernels
    for k in g_s:
        e = (g_f[k] - g_s[k]).norm() / (g_s[k].norm() + 1e-12)
        assert e < 1e-2, (k, e.item())
        e = (g_f[k] - g_r[k]).norm() / (g_r[k].norm() + 1e-12)
        assert e < 5e-2, (k, e.item())


def test_lora_wide_gpu_matches_unfused():
    from llm_fine_tune_distributed_amd.models.lora import LoRAConfig, apply_lora
    import llm_fine_tune_distributed_amd.models.transformer as T
    import llm_fine_tune_distributed_amd.ops as ops
    torch.manual_seed(0)
    cfg = tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=1024,
               vocab_size=1024, num_hidden_layers=2)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    apply_lora(m, LoRAConfig(r=16, lora_alpha=8, lora_dropout=0.1))
    for l in m.model.layers:
        for fl in (l.self_attn.lora["qkv"], l.self_attn.lora["o"], l.mlp.lora["gate_up"], l.mlp.lora["down"]):
            for bb in fl.B:
                torch.nn.init.normal_(bb, std=0.05)
    m.train()
    ids = torch.randint(0, 1024, (4, 128), device="cuda")

    def unfused(x, w, lora):
        p = lora.dropout.p if lora.training else 0.0
        seed = int(torch.randint(1, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
        x2d = x.reshape(-1, x.shape[-1])
        keep = ops.dropout_add(None, torch.ones_like(x2d), p, seed) != 0
        xd = x2d * keep / (1 - p)
        outs = [(xd.float() @ a.float().t() @ b.float().t()) for a, b in zip(lora.A, lora.B)]
        y = x2d.float() @ w.float().t() + torch.cat(outs, -1) * lora.scaling
        return y.to(x.dtype).view(*x.shape[:-1], -1)

    torch.manual_seed(7)
    out = m(ids, labels=ids)
    out.loss.backward()
    g1 = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}
    # the HIP run above took the fused MLP (gate_up GEMM with the SwiGLU epilogue, down backward returning dgu:
    # ops.lora_swiglu_mlp); the reference composes the unfused LoRA linears with the SwiGLU op (same seed order)
    orig, orig_mlp, orig_att = T.ops.lora_linear, T.ops.lora_swiglu_mlp, T.ops.lora_qkv_rope_attention
    T.ops.lora_linear = unfused
    T.ops.lora_swiglu_mlp = lambda h, wg, wd, lg, ld: unfused(ops.swiglu(unfused(h, wg, lg)), wd, ld)
    T.ops.lora_qkv_rope_attention = lambda h, w, lq, cos, sin, cu, ms, nq, nkv, hd: ops.flash_attention(
        ops.rope_(unfused(h, w, lq), cos, sin, nq, nkv, hd), cu, ms, nq, nkv, hd)
    try:
        for p in m.parameters():
            p.grad = None
        torch.manual_seed(7)
        out2 = m(ids, labels=ids)
        out2.loss.backward()
    finally:
        T.ops.lora_linear, T.ops.lora_swiglu_mlp, T.ops.lora_qkv_rope_attention = orig, orig_mlp, orig_att
    assert abs(out.loss.item() - out2.loss.item()) < 2e-2
    for n, p in m.named_parameters():
        if p.grad is not None:
            rel = (g1[n] - p.grad.float()).norm() / (p.grad.float().norm() + 1e-6)
            assert rel < 5e-2, (n, rel.item())


@pytest.mark.parametrize("r", [16, 8, 32])
def test_lora_norm_writes_widened_activation_in_place(r):
    """The RMSNorm forward writes its output into the left block of the consumer's widened activation X' (qkv /
    gate_up: add_rms_norm y_ld) and lora_fwd_inplace fills only the adapter columns: bitwise the same loss and
    gradients as the copying widening (the norm output as its own tensor, X' written by lora_fwd). r = 8 / 32 (qkv
    R = 24 / 96, outside the widening kernel's 16..64 multiples of 16): the norm writes a plain y and the copying path
    runs (no 'lora_fwd_inplace: shapes' error)."""
    from llm_fine_tune_distributed_amd.models.lora import LoRAConfig, apply_lora
    import llm_fine_tune_distributed_amd.models.transformer as T
    cfg = tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=1024,
               vocab_size=1024, num_hidden_layers=2)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    apply_lora(m, LoRAConfig(r=r, lora_alpha=8, lora_dropout=0.1))
    for l in m.model.layers:
        for fl in (l.self_attn.lora["qkv"], l.mlp.lora["gate_up"]):
            for bb in fl.B:
                torch.nn.init.normal_(bb, std=0.05)
    m.train()
    ids = torch.randint(0, 1024, (4, 128), device="cuda")
    ld = T._wide_ld(m.model.layers[0].self_attn.lora, "qkv", m.model.layers[0].self_attn.qkv_proj)
    assert ld == (640 if r == 16 else 0), ld

    def run():
        for p in m.parameters():
            p.grad = None
        torch.manual_seed(7)
        out = m(ids, labels=ids)
        out.loss.backward()
        return out.loss.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    l1, g1 = run()
    orig = T._wide_ld
    T._wide_ld = lambda *a: 0
    try:
        l2, g2 = run()
    finally:
        T._wide_ld = orig
    assert torch.equal(l1, l2) and g1.keys() == g2.keys()
    for n in g1:
        assert torch.equal(g1[n], g2[n]), n


def test_lora_wide_sync_after_edits():
    """The HIP path keeps every adapter's B inside its wide weight and its A rows in a persistent A_cat, refreshed for
    the whole model by one batched copy (ops/fused.py _wide_sync) after an optimizer epoch or an in-place edit: the
    fused forward after (a) in-place edits (version counters) and (b) raw edits + bump_param_epoch (what the flat
    optimizers do) == the unfused LoRA composition."""
    from llm_fine_tune_distributed_amd.models.lora import LoRAConfig, apply_lora
    import llm_fine_tune_distributed_amd.models.transformer as T
    import llm_fine_tune_distributed_amd.ops as ops
    torch.manual_seed(0)
    cfg = tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=1024,
               vocab_size=1024, num_hidden_layers=2)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=1)
    apply_lora(m, LoRAConfig(r=16, lora_alpha=8, lora_dropout=0.0))
    fls = [fl for l in m.model.layers
           for fl in (l.self_attn.lora["qkv"], l.self_attn.lora["o"], l.mlp.lora["gate_up"], l.mlp.lora["down"])]
    for fl in fls:
        for bb in fl.B:
            torch.nn.init.normal_(bb, std=0.05)
    m.eval()
    ids = torch.randint(0, 1024, (4, 128), device="cuda")

    def unfused(x, w, lora):
        x2d = x.reshape(-1, x.shape[-1])
        outs = [(x2d.float() @ a.float().t() @ b.float().t()) for a, b in zip(lora.A, lora.B)]
        y = x2d.float() @ w.float().t() + torch.cat(outs, -1) * lora.scaling
        return y.to(x.dtype).view(*x.shape[:-1], -1)

    def reference():
        orig, orig_mlp, orig_att = T.ops.lora_linear, T.ops.lora_swiglu_mlp, T.ops.lora_qkv_rope_attention
        T.ops.lora_linear = unfused
        T.ops.lora_swiglu_mlp = lambda h, wg, wd, lg, ld: unfused(ops.swiglu(unfused(h, wg, lg)), wd, ld)
        T.ops.lora_qkv_rope_attention = lambda h, w, lq, cos, sin, cu, ms, nq, nkv, hd: ops.flash_attention(
            ops.rope_(unfused(h, w, lq), cos, sin, nq, nkv, hd), cu, ms, nq, nkv, hd)
        try:
            with torch.no_grad():
                return m(ids, labels=ids).loss.item()
        finally:
            T.ops.lora_linear, T.ops.lora_swiglu_mlp, T.ops.lora_qkv_rope_attention = orig, orig_mlp, orig_att

    with torch.no_grad():
        l0 = m(ids, labels=ids).loss.item()
    assert abs(l0 - reference()) < 2e-2
    with torch.no_grad():  # (a) in-place edits bump the parameters' version counters
        for fl in fls:
            fl.A[0].mul_(1.5)
            fl.B[-1].add_(0.02)
        l1 = m(ids, labels=ids).loss.item()
    assert abs(l1 - l0) > 1e-3 and abs(l1 - reference()) < 2e-2
    with torch.no_grad():  # (b) raw edits (no version bump) announced by the optimizer epoch
        for fl in fls:
            fl.B[0].data.mul_(-1.0)
        ops.bump_param_epoch()
        l2 = m(ids, labels=ids).loss.item()
    assert abs(l2 - l1) > 1e-3 and abs(l2 - reference()) < 2e-2


@pytest.mark.parametrize("name,K,outs", [("qkv", 2048, [2048, 512, 512]), ("o", 2048, [2048]),
                                         ("gate_up", 2048, [11008, 11008]), ("down", 11008, [2048])])
@pytest.mark.parametrize("p", [0.0, 0.05])
def test_lora_linear_real_widths_vs_fp32(name, K, outs, p):
    """ops.lora_linear on the HIP path (padded wide weight, persistent forward GEMM, 4-wave base dgrad, lora_fwd /
    lora_bwd_dx kernels) at the SmolLM3-3B projection widths == an fp32 reference of the same LoRA math with the same
    hash dropout mask: y, dx and every adapter's dA / dB."""
    import llm_fine_tune_distributed_amd.ops as ops
    from llm_fine_tune_distributed_amd.models.lora import FusedLoRA, LoRAConfig, _widen
    torch.manual_seed(0)
    M, n = 512, sum(outs)
    owner = torch.nn.Module()
    owner.w = torch.nn.Parameter((torch.randn(n, K, device="cuda") * K ** -0.5).to(torch.bfloat16), requires_grad=False)
    fl = FusedLoRA(K, outs, [f"p{i}" for i in range(len(outs))], LoRAConfig(r=16, lora_alpha=8, lora_dropout=p),
                   [True] * len(outs), device="cuda", dtype=torch.bfloat16)
    for b in fl.B:
        torch.nn.init.normal_(b, std=0.05)
    _widen(owner, "w", fl)
    assert fl.wide.shape[1] % 128 == 0 and owner.w.data_ptr() == fl.wide.data_ptr()
    fl.train()
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
    torch.manual_seed(11)
    y = ops.lora_linear(x, owner.w, fl)
    dy = torch.randn_like(y)
    y.backward(dy)
    got = {"y": y.detach().float(), "dx": x.grad.float()}
    got.update({f"A{i}": a.grad.float() for i, a in enumerate(fl.A)})
    got.update({f"B{i}": b.grad.float() for i, b in enumerate(fl.B)})
    # fp32 reference with the kernel's dropout mask (same seed: the RNG draw order of lora_linear)
    torch.manual_seed(11)
    seed = int(torch.randint(1, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
    keep = ops.dropout_add(None, torch.ones(M, K, device="cuda", dtype=torch.bfloat16), p, seed) != 0 if p > 0 else 1
    x32 = x.detach().float().requires_grad_(True)
    As = [a.detach().float().requires_grad_(True) for a in fl.A]
    Bs = [b.detach().float().requires_grad_(True) for b in fl.B]
    xd = x32 * keep / (1 - p)
    yr = x32 @ owner.w.float().t() + torch.cat([xd @ a.t() @ b.t() for a, b in zip(As, Bs)], -1) * fl.scaling
    yr.backward(dy.float())
    want = {"y": yr.detach(), "dx": x32.grad}
    want.update({f"A{i}": a.grad for i, a in enumerate(As)})
    want.update({f"B{i}": b.grad for i, b in enumerate(Bs)})
    for k in want:
        e = ((got[k] - want[k]).norm() / (want[k].norm() + 1e-12)).item()
        assert e < 2e-2, (name, p, k, e)


