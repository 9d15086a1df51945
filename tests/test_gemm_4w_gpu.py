"""4-wave backward GEMMs (csrc/gemm_4w.hip: the 4-slot ring with one read / DMA piece per MFMA gap, wgrad_gemm /
dgrad_gemm cfg 14) against plain PyTorch fp32 references: weight gradients with and without accumulation, split-K /
hybrid pieces, gradient-norm slots, a padded x pitch; input gradients plain, on column-sliced weights, through the
wave-tail split and the hybrid split-K."""
import pytest
import torch

from llm_fine_tune_distributed_amd.ops import _ext

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _need_ext():
    assert _ext.load(), _ext.load_error()


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("cfg,T,N,K", [(14, 128, 256, 256), (14, 256, 512, 768), (14, 384, 768, 512),
                                       (14, 1024, 2304, 4352),     # 153 tiles, 8 blocks of 128 tokens
                                       (214, 512, 512, 512), (414, 1024, 256, 256), (314, 384, 512, 256),
                                       (1314, 256, 4096, 4352),    # hybrid: 256 whole tiles + 16 split 2 ways
                                       (1214, 384, 4352, 4096)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_4wave(cfg, T, N, K, accumulate):
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    out = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    base = out.float().clone()
    _ext.ops().wgrad_gemm(out, dy, x, accumulate, cfg)
    want = dy.float().t() @ x.float() + (base if accumulate else 0)
    assert rel_err(out, want) < 5e-3
    err = (out.float() - want).abs().max().item()
    assert err <= 0.02 * want.abs().max().item(), err


@pytest.mark.parametrize("cfg", [14, 214])
def test_wgrad_4wave_exact_structure(cfg):
    """Integer-valued operands (exact in fp32): a permuted token, row or column mapping anywhere in the staging,
    the transposed reads or the register epilogue changes the result bit for bit."""
    T, N, K = 256, 512, 512
    t = torch.arange(T, device=DEV)
    dy = ((t[:, None] * 3 + torch.arange(N, device=DEV)[None, :] * 7) % 5 - 2).to(torch.bfloat16)
    x = ((t[:, None] * 5 + torch.arange(K, device=DEV)[None, :] * 11) % 7 - 3).to(torch.bfloat16)
    out = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    _ext.ops().wgrad_gemm(out, dy, x, False, cfg)
    assert torch.equal(out, (dy.float().t() @ x.float()).to(torch.bfloat16))  # exact fp32 sums, one rounding


@pytest.mark.parametrize("cfg,T,N,K", [(14, 256, 512, 768), (214, 512, 512, 512), (1314, 256, 4096, 4352),
                                       (1214, 1024, 2048, 11008), (414, 1024, 2048, 2048), (214, 1024, 3072, 2048)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_4wave_norm_slots(cfg, T, N, K, accumulate):
    """Norm partials (register epilogue / split-K fixup) sum to the squared norm of the stored bf16 gradient
    (within fp32-before-rounding tolerance); slots past the capacity stay untouched."""
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    out = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    cap = -(-N // 256) * -(-K // 128) * 32
    slots = torch.zeros(cap + 64, device=DEV)
    slots[cap:] = 7.0
    # garbage in the caching allocator's free blocks: a hybrid launch parks the whole tiles' slots in an
    # uninitialised split-K buffer, every one of them must be written
    torch.full((1 << 26,), float("nan"), device=DEV)
    _ext.ops().wgrad_gemm(out, dy, x, accumulate, cfg, slots[:cap])
    want = out.float().pow(2).sum().item()
    assert abs(slots[:cap].sum().item() - want) <= 1e-3 * want
    assert torch.all(slots[cap:] == 7.0)


@pytest.mark.parametrize("cfg", [414, 1214])
def test_wgrad_4wave_matches_ring_split_exactly(cfg):
    """Split pieces (414: 4 equal token ranges per tile; 1214: the hybrid split) are whole 128-token blocks summed in a
    fixed order: repeated launches are bitwise identical (deterministic), and the result matches the fp32 reference."""
    torch.manual_seed(3)
    T, N, K = 1024, 512, 768
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    o1 = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    _ext.ops().wgrad_gemm(o1, dy, x, False, cfg)
    _ext.ops().wgrad_gemm(o2, dy, x, False, cfg)
    assert torch.equal(o1, o2)
    assert rel_err(o1, dy.float().t() @ x.float()) < 5e-3


@pytest.mark.parametrize("M,K,N,wpad", [(256, 128, 256, 0), (512, 2048, 768, 0), (256, 384, 512, 64),
                                        (768, 1024, 256, 0), (2048, 11008, 2048, 0)])
@pytest.mark.parametrize("cfg", [14])
def test_dgrad_4wave_plain(M, K, N, wpad, cfg):
    torch.manual_seed(0)
    dy = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    wfull = torch.randn(K, N + wpad, device=DEV, dtype=torch.bfloat16)
    w = wfull[:, :N]
    out = _ext.ops().dgrad_gemm(dy, w, None, cfg)
    assert out.shape == (M, N)
    assert rel_err(out, dy.float() @ w.float()) < 5e-3
    # asymmetric structure: a column-shifted identity catches any transposed / permuted mapping (exact)
    eye = torch.zeros(K, N, device=DEV)
    eye[torch.arange(min(K, N)), (torch.arange(min(K, N)) + 5) % N] = 1.0
    ramp = (torch.arange(M * K, device=DEV) % 251).float().view(M, K).to(torch.bfloat16)
    got = _ext.ops().dgrad_gemm(ramp, eye.to(torch.bfloat16), None, cfg).float()
    assert torch.equal(got, ramp.float() @ eye)


def test_dgrad_4wave_refuses_the_swiglu_epilogue():
    """The SwiGLU-backward epilogue runs on cfg 7 (its LDS-staged epilogue: 0.425 vs 0.483 ms for the 4-wave kernel's
    register epilogue, profiles/r6_gemm_routing.md); the 4-wave kernel refuses it instead of computing a plain dX."""
    dy = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    gu = torch.randn(256, 512, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _ext.ops().dgrad_gemm(dy, w, gu, 14)


@pytest.mark.parametrize("cfg,swiglu", [(14, False), (7, True), (7, False)])
def test_dgrad_4wave_wave_tail(swiglu, cfg, monkeypatch):
    """SmolLM3 down projection grid (43 x 32 tiles = 5.375 rounds): the whole rounds on the 4-wave kernel (or cfg 7
    with the SwiGLU backward) + the leftover columns as 256 x 128 half tiles of the ring kernel (SFTAMD_DGRAD_TAIL=2)
    == the fp32 reference."""
    torch.manual_seed(2)
    M, K, N = 8192, 128, 11008
    dy = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(K, N, device=DEV)).to(torch.bfloat16)
    gu = torch.randn(M, 2 * N, device=DEV, dtype=torch.bfloat16) if swiglu else None
    dact = dy.float() @ w.float()
    if swiglu:
        g, u = gu.float().chunk(2, dim=-1)
        s = torch.sigmoid(g)
        want = torch.cat([dact * u * s * (1 + g * (1 - s)), dact * g * s], dim=-1)
    else:
        want = dact
    for tail in ("0", "2"):
        monkeypatch.setenv("SFTAMD_DGRAD_TAIL", tail)
        got = _ext.ops().dgrad_gemm(dy, w, gu, cfg)
        assert rel_err(got, want) < 1e-2, tail


@pytest.mark.parametrize("cfg", [14])
@pytest.mark.parametrize("M,K,N", [(10240, 1024, 2048), (2560, 4096, 2048), (4352, 512, 4096)])
def test_dgrad_4wave_hybrid_splitk(M, K, N, cfg):
    """Grids that are not whole rounds of 256 workgroups (the recipe's padding-free M = 10240: 320 tiles) run the
    whole rounds as whole tiles and split the leftover tiles over the reduction (fp32 slabs + ordered fixup):
    == the fp32 reference, deterministic, and exact on integer data."""
    torch.manual_seed(5)
    dy = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(K, N, device=DEV)).to(torch.bfloat16)
    out = _ext.ops().dgrad_gemm(dy, w, None, cfg)
    assert rel_err(out, dy.float() @ w.float()) < 5e-3
    assert torch.equal(out, _ext.ops().dgrad_gemm(dy, w, None, cfg))
    ramp = (torch.arange(M * K, device=DEV) % 7 - 3).float().view(M, K).to(torch.bfloat16)
    wi = (torch.arange(K * N, device=DEV) % 5 - 2).float().view(K, N).to(torch.bfloat16)
    got = _ext.ops().dgrad_gemm(ramp, wi, None, cfg)
    assert torch.equal(got, (ramp.float() @ wi.float()).to(torch.bfloat16))


@pytest.mark.parametrize("cfg,T,N,K", [(14, 512, 22016 // 86 * 2, 2048), (14, 1024, 512, 768), (1214, 1024, 2048, 11008 // 256 * 256)])
def test_wgrad_4wave_padded_x_pitch(cfg, T, N, K):
    """x [T, K] as a view into a wider buffer (padded row pitch, e.g. the gate_up input written by the norm with
    y_ld): bitwise the same dW (and norm slots) as from a contiguous x."""
    torch.manual_seed(1)
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    buf = torch.randn(T, K + 64, device=DEV, dtype=torch.bfloat16)
    buf[:, :K] = x
    cap = -(-N // 256) * -(-K // 128) * 32
    o1, o2 = torch.empty(N, K, device=DEV, dtype=torch.bfloat16), torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    s1, s2 = torch.zeros(cap, device=DEV), torch.zeros(cap, device=DEV)
    _ext.ops().wgrad_gemm(o1, dy, x, False, cfg, s1)
    _ext.ops().wgrad_gemm(o2, dy, buf[:, :K], False, cfg, s2)
    assert torch.equal(o1, o2) and torch.equal(s1, s2)


@pytest.mark.parametrize("M,K,N", [(256, 256, 256), (1024, 2048, 2048), (8192, 2048, 2048), (512, 4096, 4096)])
def test_dgrad_4wave_attention_delta(M, K, N):
    """dgrad_gemm_delta (the o_proj input gradient with flash attention's delta in the epilogue): dO bitwise the plain
    4-wave dgrad, delta [N / 128, M] == per-head rowsum(dO . a) in fp32, and exact on integer data (a head / row
    mix-up cannot hide)."""
    torch.manual_seed(7)
    dy = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(K, N, device=DEV)).to(torch.bfloat16)
    a = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    dx, delta = _ext.ops().dgrad_gemm_delta(dy, w, a)
    assert torch.equal(dx, _ext.ops().dgrad_gemm(dy, w, None, 14))
    assert delta.shape == (N // 128, M) and delta.dtype == torch.float32 and delta.is_contiguous()
    want = (dx.float() * a.float()).view(M, N // 128, 128).sum(-1).t()
    assert (delta - want).abs().max().item() <= 1e-5 * want.abs().max().item() + 1e-6
    ramp = (torch.arange(M * K, device=DEV) % 7 - 3).float().view(M, K).to(torch.bfloat16)
    eye = torch.zeros(K, N, device=DEV)
    eye[torch.arange(min(K, N)), (torch.arange(min(K, N)) + 5) % N] = 1.0
    ai = ((torch.arange(M * N, device=DEV) * 13) % 5 - 2).float().view(M, N).to(torch.bfloat16)
    dxi, di = _ext.ops().dgrad_gemm_delta(ramp, eye.to(torch.bfloat16), ai)
    exp = ramp.float() @ eye
    assert torch.equal(dxi.float(), exp)
    assert torch.equal(di, (exp * ai.float()).view(M, N // 128, 128).sum(-1).t())


def test_dgrad_4wave_attention_delta_refuses_split_shapes():
    """The delta epilogue runs on whole tiles only: a reduction long enough for the hybrid split-K is refused."""
    dy = torch.randn(256, 8192, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(8192, 512, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _ext.ops().dgrad_gemm_delta(dy, w, torch.randn(256, 512, device=DEV, dtype=torch.bfloat16))


def test_4wave_grids_under_a_cu_budget():
    """set_cu_budget(248) (collectives holding CUs at N > 1, profiles/r6_cu_contention.md): a 256-tile input gradient
    with a short reduction splits its leftover 8 tiles over K, the hybrid weight gradient whole-rounds 248 tiles; both
    == the fp32 reference and deterministic; the delta epilogue still runs on whole tiles (no split)."""
    from llm_fine_tune_distributed_amd import ops
    torch.manual_seed(11)
    try:
        assert ops.set_cu_budget(248) == 248
        dy = torch.randn(4096, 2048, device=DEV, dtype=torch.bfloat16)
        w = (0.05 * torch.randn(2048, 4096, device=DEV)).to(torch.bfloat16)
        _ext.ops().dispatch_trace(True)
        try:
            out = _ext.ops().dgrad_gemm(dy, w, None, 14)
        finally:
            _ext.ops().dispatch_trace(False)
        assert "dgrad.splitk" in _ext.ops().dispatch_trace_read()
        assert rel_err(out, dy.float() @ w.float()) < 5e-3
        assert torch.equal(out, _ext.ops().dgrad_gemm(dy, w, None, 14))
        a = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
        dx, delta = _ext.ops().dgrad_gemm_delta(dy, w, a)
        assert rel_err(dx, dy.float() @ w.float()) < 5e-3
        want = (dx.float() * a.float()).view(4096, 32, 128).sum(-1).t()
        assert (delta - want).abs().max().item() <= 1e-5 * want.abs().max().item() + 1e-6
        T, N, K = 1024, 2048, 11008 // 256 * 256  # 8 x 43 = 344 tiles: 248 whole + 96 split 2 ways
        dyw = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
        x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
        o = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
        _ext.ops().wgrad_gemm(o, dyw, x, False, 1214)
        assert rel_err(o, dyw.float().t() @ x.float()) < 5e-3
    finally:
        ops.set_cu_budget(0)
    assert ops.cu_budget() == 256


@pytest.mark.parametrize("N0,K0,N1,K1,T", [(2048, 10752, 5632, 2048, 256),    # 336 + 176 = 512 tiles: 2 whole rounds
                                           (2048, 11008, 22016, 2048, 256),   # the SmolLM3 MLP: 1032 = 4 rounds + 8
                                           (2048, 11008, 22016, 2048, 1024)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_pair_one_launch(N0, K0, N1, K1, T, accumulate):
    """wgrad_gemm_pair (the MLP's down + gate_up weight gradients as one grid) == two cfg-14 launches: whole tiles
    bitwise, the split leftover tiles of problem 1 within fp32-order rounding, deterministic; the norm slots sum to
    the squared norm of what was stored."""
    torch.manual_seed(13)
    dy0 = torch.randn(T, N0, device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(T, K0, device=DEV, dtype=torch.bfloat16)
    dy1 = torch.randn(T, N1, device=DEV, dtype=torch.bfloat16)
    x1 = torch.randn(T, K1, device=DEV, dtype=torch.bfloat16)
    base0 = torch.randn(N0, K0, device=DEV, dtype=torch.bfloat16)
    base1 = torch.randn(N1, K1, device=DEV, dtype=torch.bfloat16)
    w0, w1 = base0.clone(), base1.clone()
    r0, r1 = base0.clone(), base1.clone()
    cap0 = (N0 // 256) * (K0 // 128) * 32
    cap1 = (N1 // 256) * (K1 // 128) * 32
    n0 = torch.zeros(cap0, device=DEV)
    n1 = torch.zeros(cap1, device=DEV)
    _ext.ops().wgrad_gemm_pair(w0, dy0, x0, accumulate, n0, w1, dy1, x1, accumulate, n1)
    _ext.ops().wgrad_gemm(r0, dy0, x0, accumulate, 14)
    _ext.ops().wgrad_gemm(r1, dy1, x1, accumulate, 14)
    assert torch.equal(w0, r0)
    tiles = (N0 // 256) * (K0 // 256) + (N1 // 256) * (K1 // 256)
    if tiles % 256 == 0:
        assert torch.equal(w1, r1)
    else:
        assert rel_err(w1, r1) < 1e-2
        assert (w1 != r1).float().mean().item() < 0.05  # only the split leftover tiles may differ
    want = (dy1.float().t() @ x1.float()) + (base1.float() if accumulate else 0)
    assert rel_err(w1, want) < 5e-3
    assert abs(n0.sum().item() - w0.float().pow(2).sum().item()) < 1e-3 * w0.float().pow(2).sum().item()
    assert abs(n1.sum().item() - w1.float().pow(2).sum().item()) < 1e-3 * w1.float().pow(2).sum().item()
    v0, v1 = base0.clone(), base1.clone()
    _ext.ops().wgrad_gemm_pair(v0, dy0, x0, accumulate, None, v1, dy1, x1, accumulate, None)
    assert torch.equal(v0, w0) and torch.equal(v1, w1)


def test_wgrad_pair_refuses_a_leftover_in_the_first_problem():
    """The partial last round must fall in the second problem (its fixup); a pair whose leftover tiles would reach into
    the first one is refused (ops.fused._pair_ok routes such pairs to two launches)."""
    dy0 = torch.randn(256, 22016, device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(256, 2048, device=DEV, dtype=torch.bfloat16)
    dy1 = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    x1 = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    o0 = torch.empty(22016, 2048, device=DEV, dtype=torch.bfloat16)
    o1 = torch.empty(256, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _ext.ops().wgrad_gemm_pair(o0, dy0, x0, False, None, o1, dy1, x1, False, None)


@pytest.mark.parametrize("T", [1024, 8192])
def test_wgrad_pair_split_all(T):
    """o_proj + qkv weight gradients as one launch with every tile split 3 ways (split_all): == two cfg-14 launches
    within fp32-order rounding, == the fp32 reference, deterministic, norm slots sum to the stored squared norm."""
    torch.manual_seed(17)
    dy0 = torch.randn(T, 2048, device=DEV, dtype=torch.bfloat16)
    x0 = torch.randn(T, 2048, device=DEV, dtype=torch.bfloat16)
    dy1 = torch.randn(T, 3072, device=DEV, dtype=torch.bfloat16)
    x1 = torch.randn(T, 2048, device=DEV, dtype=torch.bfloat16)
    w0 = torch.empty(2048, 2048, device=DEV, dtype=torch.bfloat16)
    w1 = torch.empty(3072, 2048, device=DEV, dtype=torch.bfloat16)
    n0 = torch.zeros(8 * 16 * 32, device=DEV)
    n1 = torch.zeros(12 * 16 * 32, device=DEV)
    _ext.ops().wgrad_gemm_pair(w0, dy0, x0, False, n0, w1, dy1, x1, False, n1, 3)
    assert rel_err(w0, dy0.float().t() @ x0.float()) < 5e-3
    assert rel_err(w1, dy1.float().t() @ x1.float()) < 5e-3
    r0, r1 = torch.empty_like(w0), torch.empty_like(w1)
    _ext.ops().wgrad_gemm(r0, dy0, x0, False, 14)
    _ext.ops().wgrad_gemm(r1, dy1, x1, False, 14)
    assert rel_err(w0, r0) < 1e-2 and rel_err(w1, r1) < 1e-2
    for n, w in ((n0, w0), (n1, w1)):
        ref = w.float().pow(2).sum().item()
        assert abs(n.sum().item() - ref) < 1e-3 * ref
    v0, v1 = torch.empty_like(w0), torch.empty_like(w1)
    _ext.ops().wgrad_gemm_pair(v0, dy0, x0, False, None, v1, dy1, x1, False, None, 3)
    assert torch.equal(v0, w0) and torch.equal(v1, w1)


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("split_left", [0, 3])
def test_wgrad_multi_four_problems(accumulate, split_left):
    """wgrad_gemm_multi: a layer's down + gate_up with the next layer's o_proj + qkv as ONE grid (SmolLM3 widths,
    1192 tiles = 4 whole rounds + 168 tiles split over the tokens, spanning three problems): every gradient == the
    fp32 reference, the whole tiles == separate cfg-14 launches bitwise, deterministic, norm slots sum to the stored
    squared norm per problem."""
    torch.manual_seed(19)
    T = 8192
    shapes = [(2048, 11008), (22016, 2048), (2048, 2048), (3072, 2048)]  # (N, K): down, gate_up, o, qkv
    dys = [(0.05 * torch.randn(T, n, device=DEV)).to(torch.bfloat16) for n, _ in shapes]
    xs = [(0.05 * torch.randn(T, k, device=DEV)).to(torch.bfloat16) for _, k in shapes]
    bases = [torch.randn(n, k, device=DEV, dtype=torch.bfloat16) for n, k in shapes]
    outs = [b.clone() for b in bases]
    norms = [torch.zeros((n // 256) * (k // 128) * 32, device=DEV) for n, k in shapes]
    acc = [1 if accumulate else 0] * 4
    _ext.ops().wgrad_gemm_multi(outs, dys, xs, acc, norms, 0, split_left)
    for o, dy, x, b, nr in zip(outs, dys, xs, bases, norms):
        want = dy.float().t() @ x.float() + (b.float() if accumulate else 0)
        assert rel_err(o, want) < 5e-3
        ref = o.float().pow(2).sum().item()
        assert abs(nr.sum().item() - ref) < 1e-3 * ref
    # down (problem 0) lies wholly in the 4 whole rounds: bitwise the single cfg-14 launch
    r0 = bases[0].clone()
    _ext.ops().wgrad_gemm(r0, dys[0], xs[0], accumulate, 14)
    assert torch.equal(outs[0], r0)
    again = [b.clone() for b in bases]
    empty = torch.empty(0, device=DEV)
    _ext.ops().wgrad_gemm_multi(again, dys, xs, acc, [empty] * 4, 0, split_left)
    assert all(torch.equal(a, o) for a, o in zip(again, outs))


def test_wgrad_multi_three_problems_small():
    """Three problems below one round with every tile split (split_all) and the hybrid rule on a ragged total."""
    torch.manual_seed(23)
    T = 1024
    shapes = [(512, 256), (256, 512), (768, 256)]
    dys = [torch.randn(T, n, device=DEV, dtype=torch.bfloat16) for n, _ in shapes]
    xs = [torch.randn(T, k, device=DEV, dtype=torch.bfloat16) for _, k in shapes]
    empty = torch.empty(0, device=DEV)
    for split_all in (2, 4):
        outs = [torch.empty(n, k, device=DEV, dtype=torch.bfloat16) for n, k in shapes]
        _ext.ops().wgrad_gemm_multi(outs, dys, xs, [0, 0, 0], [empty] * 3, split_all, 0)
        for o, dy, x in zip(outs, dys, xs):
            assert rel_err(o, dy.float().t() @ x.float()) < 5e-3
