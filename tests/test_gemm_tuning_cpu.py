"""The forward-GEMM routing set read from the TunableOp file (utils/gemm_tuning._tuned_tn): only bf16 TN rows with
the contiguous leading dimensions count."""
from llm_fine_tune_distributed_amd.utils.gemm_tuning import _tuned_tn


def test_tuned_tn_keeps_only_contiguous_bf16_tn_rows(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text(
        "Validator,PT_VERSION,2.10.0\n"
        "GemmTunableOp_BFloat16_TN,tn_3072_8192_2048_ld_2048_2048_3072,Gemm_Rocblas_1,0.04\n"
        "GemmTunableOp_Half_TN,tn_2048_8192_2048_ld_2048_2048_2048,Gemm_Hipblaslt_2,0.03\n"
        "GemmTunableOp_float_TN,tn_4096_8192_2048_ld_2048_2048_4096,Gemm_Hipblaslt_3,0.03\n"
        "GemmTunableOp_BFloat16_NN,nn_2048_8192_3072_ld_2048_3072_2048,Gemm_Rocblas_4,0.05\n"
        "GemmTunableOp_BFloat16_TN,tn_2048_8192_11008_ld_11136_11008_2048,Gemm_Rocblas_5,0.1\n"
        "GemmTunableOp_BFloat16_TN,tn_bad_row\n")
    assert _tuned_tn(str(p)) == frozenset({(3072, 8192, 2048)})


def test_tuned_tn_missing_file_is_empty(tmp_path):
    assert _tuned_tn(str(tmp_path / "none.csv")) == frozenset()


def test_shipped_selections_cover_the_headline_shapes():
    import os
    from llm_fine_tune_distributed_amd.utils import gemm_tuning
    shapes = _tuned_tn(gemm_tuning._DEFAULT)
    assert os.path.exists(gemm_tuning._DEFAULT)
    assert all(len(s) == 3 for s in shapes)


def test_wgrad_routing_under_a_cu_budget(monkeypatch):
    """The split decisions of the 4-wave weight gradients follow the CU budget (ops.set_cu_budget): o_proj's 64 tiles
    split 3 ways (192 workgroups) instead of 4 (256) when 8 CUs are reserved; the other SmolLM3 shapes keep theirs."""
    import llm_fine_tune_distributed_amd.ops.fused as F
    shapes = {"o": (2048, 2048), "qkv": (3072, 2048), "down": (2048, 11008), "lm_head": (128256, 2048),
              "gate_up": (22016, 2048)}
    monkeypatch.setattr(F, "_WGRAD_MODE", "auto")
    monkeypatch.setattr(F, "_CU_BUDGET", 256)
    assert {k: F._wgrad_cfg(8192, n, kk) for k, (n, kk) in shapes.items()} == {
        "o": 414, "qkv": 214, "down": 1214, "lm_head": 1214, "gate_up": 14}
    monkeypatch.setattr(F, "_CU_BUDGET", 248)
    assert {k: F._wgrad_cfg(8192, n, kk) for k, (n, kk) in shapes.items()} == {
        "o": 314, "qkv": 214, "down": 1214, "lm_head": 1214, "gate_up": 14}


def test_weight_gradient_pair_planning():
    """Pair planning (ops.fused): pairs smaller than one round split every tile s ways (o_proj + qkv: 64 + 96 tiles ->
    3 ways, 2 rounds of third-tiles); larger pairs run whole rounds + the split leftover (0); CPU tensors never pair."""
    import torch
    import llm_fine_tune_distributed_amd.ops.fused as F
    assert F._pair_split(64, 96, 8192) == 3
    assert F._pair_split(344, 688, 8192) == 0 and F._pair_split(256, 384, 8192) == 0
    assert F._pair_split(64, 96, 256) == 2  # at most T / 128 pieces per tile
    p0 = torch.nn.Parameter(torch.zeros(256, 256))
    p1 = torch.nn.Parameter(torch.zeros(256, 256))
    x = torch.zeros(1024, 256, dtype=torch.bfloat16)
    assert not F._pair_ok(p0, x, x, p1, x, x)


def test_dgrad_routing():
    """Input-gradient configs (ops.fused._dgrad_cfg): the 8-wave 32-deep ring (5) for the SwiGLU-fused down dgrad and
    for plain dgrads whose grid is whole rounds or takes the wave-tail launch; the 4-wave ring (14) for the
    vocabulary-long lm_head reduction, ragged token counts and under SFTAMD_DGRAD_RING8=0."""
    import torch
    import llm_fine_tune_distributed_amd.ops.fused as F

    def cfg(M, K, N, swiglu=False):
        return F._dgrad_cfg(torch.empty(M, K, device="meta"), swiglu=swiglu, N=N)

    assert cfg(8192, 2048, 11008, swiglu=True) == 5  # down + SwiGLU backward (1376 tiles, wave tail)
    assert cfg(8192, 22016, 2048) == 5 and cfg(8192, 3072, 2048) == 5 and cfg(8192, 2048, 2048) == 5
    assert cfg(8192, 2048, 11008) == 5  # 1376 tiles: 5 rounds + the half-tile round
    assert cfg(8192, 128256, 2048) == 14  # lm_head
    assert cfg(8192 + 512, 2048, 2048) == 14  # 34 x 8 = 272 tiles: 256 % 34 != 0, no wave tail
    assert cfg(2048, 2048, 2048) == 14  # 64 tiles: less than one round
    assert cfg(8192, 2016, 2048) == 5 and cfg(8192, 1984, 2048) == 7  # K % 128 != 0
    F_ring8 = F._DGRAD_RING8
    try:
        F._DGRAD_RING8 = False
        assert cfg(8192, 22016, 2048) == 14
    finally:
        F._DGRAD_RING8 = F_ring8


def test_attention_wgrad_carry_into_the_previous_mlp_launch():
    """The cross-layer hand-off (ops.fused wgrad_carry_scope): the leftover split of a four-problem launch (1192
    SmolLM3 tiles -> unsplit; Llama's 3328 tiles are whole rounds -> 1), a scope hands one MLP dict to the next
    attention only, an armed dict takes the o_proj + qkv jobs and the MLP side then accumulates all four gradients
    (CPU: the per-job fallback), and no carry outside a scope."""
    import torch
    import llm_fine_tune_distributed_amd.ops.fused as F
    assert F._multi_split(344 + 688 + 64 + 96, 8192) == 1  # 168 left over: an unsplit partial round is cheapest
    assert F._multi_split(4 * 256 + 40, 8192) == 6  # a small leftover is split to fill the round
    assert F._multi_split(1792 + 896 + 384 + 256, 8192) == 1
    assert F._carry_take() is None
    with F.wgrad_carry_scope(True):
        box = {"armed": True}
        F._carry_put(box)
        assert F._carry_take() is box and F._carry_take() is None
        F._carry_put({})  # an MLP whose gate_up backward will not run (unarmed) is never offered
        assert F._carry_take() is None
    assert F._CARRY is None
    torch.manual_seed(0)
    T = 64

    def job(n, k):
        p = torch.nn.Parameter(torch.zeros(n, k))
        p.main_grad = torch.zeros(n, k)
        p._sftamd_fresh = True
        return p, torch.randn(T, n), torch.randn(T, k)

    o, qkv, down, gu = job(8, 16), job(24, 16), job(16, 32), job(64, 16)
    carry = {"armed": True}
    F._carry_or_launch(carry, [o, qkv])
    assert carry["attn"] == [o, qkv] and o[0].main_grad.abs().sum() == 0  # deferred, nothing computed yet
    F._accumulate_weight_grad_jobs([down, gu] + carry.pop("attn"))
    for p, dy, x in (o, qkv, down, gu):
        assert torch.allclose(p.main_grad, dy.t() @ x, atol=1e-4)
    F._carry_or_launch(None, [o, qkv])  # no carry: launched at once (accumulating now)
    assert torch.allclose(o[0].main_grad, 2 * (o[1].t() @ o[2]), atol=1e-4)
