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


# Per-parameter relative gradient error bounds, ~2x the maxima measured on MI355X (tools/gpu_runs/r5_run03.sh:
# profiles/r5_default_path_errors.md). The errors come from bf16 activations (every parameter of a class sits at about
# the same value), so a kernel bug touching a few percent of a weight's rows or columns stands far above them.
SMOLLM3_BOUNDS = [("model.norm", 1.6e-2), ("layernorm", 4e-2), ("mlp", 4e-2), ("self_attn", 3.6e-2),
                  ("embed", 3.6e-2)]
LLAMA_BOUNDS = [("model.norm", 2.1e-2), ("input_layernorm", 8e-2), ("qkv", 8e-2), ("o_proj", 6e-2),
                ("post_attention_layernorm", 5.5e-2), ("mlp", 5.4e-2), ("embed", 5.4e-2), ("lm_head", 4e-2)]


def _cfg():
    return tiny("smollm3", hidden_size=2048, num_attention_heads=16, num_key_value_heads=4, head_dim=128,
                intermediate_size=11008, vocab_size=8192, num_hidden_layers=4, max_position_embeddings=4096,
                rope_theta=2e6)


def _report(tag, errs, tr=None):
    """DEFAULT_PATH_REPORT=<file>: append the per-parameter relative gradient errors (how the bounds were set) and the
    dispatch trace."""
    import json
    import os
    path = os.environ.get("DEFAULT_PATH_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": tag, "errors": errs, "trace": tr}) + "\n")


def _run_vs_reference(cfg, monkeypatch, B=16, T=512):
    """Default-path fwd + bwd (dispatch trace on) and the fp32 PyTorch reference with the same weights.
    Returns (trace, loss, ref loss, {param: relative grad error}, fused clip norm^2, reference norm^2)."""
    from llm_fine_tune_distributed_amd.parallel.ddp import DDPEngine
    from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
    assert _ext.load(), _ext.load_error()
    enable_tuned_gemms()  # as SFTTrainer does (SFTConfig.gemm_tuning): the shipped hipBLASLt selections
    torch.manual_seed(0)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=11)
    ref = build_model(cfg, device="cuda", dtype=torch.float32, seed=11)
    with torch.no_grad():
        for (n, p), (n2, q) in zip(m.named_parameters(), ref.named_parameters()):
            assert n == n2
            q.copy_(p.float())
    ids = torch.randint(0, cfg.vocab_size, (B, T), device="cuda")
    labels = ids.clone()
    labels[:, T - T // 5:] = -100  # padded-batch style ignored tail

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
    monkeypatch.setenv("SFTAMD_DISABLE_HIP", "1")
    ref.train()
    out_r = ref(ids, labels=labels)
    out_r.loss.backward()
    monkeypatch.delenv("SFTAMD_DISABLE_HIP")
    gref = {n: p.grad.float() for n, p in ref.named_parameters()}
    errs, total_ref = {}, 0.0
    for p, _, _, _ in eng.layout:
        name = eng.param_names[id(p)]
        g = p.main_grad.float()
        errs[name] = ((g - gref[name]).norm() / (gref[name].norm() + 1e-12)).item()
        total_ref += gref[name].pow(2).sum().item()
    assert norm2 is not None
    return tr, out.loss.item(), out_r.loss.item(), errs, norm2.item(), total_ref


def _check_errors(errs, bounds):
    """bounds: (substring, max relative error) pairs, first match wins — about 2x the maxima measured on MI355X."""
    for name, e in errs.items():
        lim = next(b for key, b in bounds if key in name)
        assert e < lim, (name, e, lim)


def test_default_path_smollm3_widths_vs_fp32_reference(monkeypatch):
    cfg = _cfg()
    tr, loss, loss_r, errs, norm2, total_ref = _run_vs_reference(cfg, monkeypatch)
    _report("smollm3", errs, tr)
    # ---- which variants ran (the defaults of ops/fused.py and the C++ launchers at these shapes)
    assert tr.get("tn.rope.c11", 0) == 3 and tr.get("tn.rope.tail", 0) == 3, tr  # qkv + RoPE, 384-tile tail split
    # plain forwards: hipBLASLt for the shapes with a TunableOp selection (SmolLM3 widths at 8192 tokens), the
    # row-contiguous kernel for the rest — here only the lm_head of the reduced 8192-token vocabulary
    assert tr.get("tn.c60", 0) == 1, tr
    assert tr.get("attn.fwd32", 0) == 4 and tr.get("attn.dkdv32", 0) == 4 and tr.get("attn.dq32", 0) == 4, tr
    assert tr.get("attn.bwd_rope_epi", 0) == 3, tr  # inverse RoPE in the dq / dK epilogues of the 3 RoPE layers
    # wgrad: the 4-wave ring (csrc/gemm_4w.hip) for the 8192-vocab lm_head (256 tiles); the MLP's down + gate_up as
    # ONE launch per layer (344 + 688 tiles, the 8 leftover tiles split) and o_proj + qkv as one (64 + 96 tiles split 3
    # ways; the NoPE layer's through its qkv node); no 8-wave ring, no lone o_proj / qkv launch
    assert tr.get("wgrad.c14", 0) > 0, tr
    # (with each layer's o_proj + qkv carried into the previous layer's MLP launch: layers 1..3's attention join
    # MLP 0..2 as four-problem grids; layer 0's attention and layer 3's MLP stay pairs)
    assert tr.get("wgrad.multi4", 0) == 3 and tr.get("wgrad.pair", 0) == 2, tr
    assert "wgrad.c214" not in tr and "wgrad.c414" not in tr, tr
    assert not any(k in tr for k in ("wgrad.c9", "wgrad.c10", "wgrad.c209", "wgrad.c210")), tr
    assert tr.get("wgrad.norm_slots", 0) > 0, tr
    assert tr.get("dgrad.swiglu.c5", 0) >= 4 and tr.get("dgrad.tail", 0) > 0, tr  # down dgrad + SwiGLU bwd
    # gate_up (K = 22016) x 4 + lm_head (8192-token vocabulary) + qkv x 4: whole rounds of 256 tiles on the 8-wave
    # 32-deep ring; o_proj x 4 on the 4-wave kernel with flash attention's delta in the epilogue (RoPE and NoPE
    # layers), so no standalone delta kernel
    assert tr.get("dgrad.c5", 0) >= 9 and "dgrad.c14" not in tr and "dgrad.c12" not in tr, tr
    assert tr.get("dgrad.c14.delta", 0) == 4 and "attn.delta_kernel" not in tr, tr
    assert "attn.dq3" not in tr, tr  # (the recompute path: past the dS^T budget only)
    # ---- numerics vs the fp32 reference path (same weights, PyTorch ops)
    assert abs(loss - loss_r) < 2e-2 * abs(loss_r)
    _check_errors(errs, SMOLLM3_BOUNDS)
    # the clip norm from the wgrad-epilogue slots + the leftover pass == the reference gradient norm
    assert abs(norm2 ** 0.5 - total_ref ** 0.5) < 3e-2 * total_ref ** 0.5


def test_default_path_llama3_8b_widths_vs_fp32_reference(monkeypatch):
    """BASELINE config 5's architecture at its real widths (hidden 4096, intermediate 14336 -> gate_up 28672, 32 q / 8
    kv heads x 128, every layer RoPE, untied head), 4 layers, 8192-token vocabulary, 16 x 512 tokens: the default
    dispatch at those shapes and every gradient vs the fp32 reference."""
    from llm_fine_tune_distributed_amd.models.config import llama3_8b
    cfg = llama3_8b()
    cfg.num_hidden_layers = 4
    cfg.vocab_size = 8192
    cfg.eos_token_id = 2
    tr, loss, loss_r, errs, norm2, total_ref = _run_vs_reference(cfg, monkeypatch)
    _report("llama3_8b", errs, tr)
    assert tr.get("attn.fwd32", 0) == 4 and tr.get("attn.dkdv32", 0) == 4 and tr.get("attn.dq32", 0) == 4, tr
    assert tr.get("attn.bwd_rope_epi", 0) == 4, tr  # every Llama layer is a RoPE layer
    # qkv + RoPE: 32 x 24 = 768 tiles = 3 whole rounds, so no 256 x 128 tail launch
    assert tr.get("tn.rope.c11", 0) == 4 and "tn.rope.tail" not in tr, tr
    # o / gate_up / down at 8192 tokens have TunableOp selections (hipBLASLt / rocBLAS, 49.6 vs 48.3 samples/s for the
    # row-contiguous kernel in the 8B bench); the reduced-vocabulary lm_head has none: the row-contiguous kernel
    assert tr.get("tn.c60", 0) == 1, tr
    assert tr.get("wgrad.c14", 0) > 0, tr  # wgrad: lm_head (4-wave ring, 512 tiles)
    # down + gate_up (896 + 1792 tiles) and o + qkv (256 + 384) as one launch each per layer
    # (1792 + 896 + 384 + 256 tiles = 13 whole rounds per four-problem grid)
    assert tr.get("wgrad.multi4", 0) == 3 and tr.get("wgrad.pair", 0) == 2, tr
    assert tr.get("wgrad.norm_slots", 0) > 0, tr
    assert tr.get("dgrad.swiglu.c5", 0) == 4, tr  # down dgrad + SwiGLU bwd: 56 x 32 tiles = 7 whole rounds
    # gate_up (K = 28672), lm_head, qkv: whole rounds on the 8-wave 32-deep ring
    assert tr.get("dgrad.c5", 0) >= 9 and "dgrad.c14" not in tr and "dgrad.c12" not in tr, tr
    assert tr.get("dgrad.c14.delta", 0) == 4 and "attn.delta_kernel" not in tr, tr  # o_proj + the attention delta
    assert abs(loss - loss_r) < 2e-2 * abs(loss_r)
    _check_errors(errs, LLAMA_BOUNDS)
    assert abs(norm2 ** 0.5 - total_ref ** 0.5) < 3e-2 * total_ref ** 0.5
