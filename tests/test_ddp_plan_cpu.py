"""xGMI bucket plan and oversized-parameter splitting of the DDP engine."""
import pytest
import torch

from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.parallel.ddp import DDPEngine, plan_bucket_mb


def test_plan_grows_with_world_size_and_is_clamped():
    caps = [plan_bucket_mb(n) for n in (1, 2, 4, 8)]
    assert caps == sorted(caps) and caps[0] < 20 and 100 < caps[3] <= 256
    assert plan_bucket_mb(8, total_bytes=64 * 2 ** 20) == 16.0  # tiny models still get >= 8 buckets (floor 16)
    assert plan_bucket_mb(8, alpha_us=1000, link_gbps=1000) == 256.0


@pytest.mark.parametrize("world", [1, 2, 8])
def test_oversized_param_split_layout_and_ready_signalling(world):
    m = build_model(tiny(), dtype=torch.float32, seed=0)
    eng = DDPEngine(m, world_size=world, rank=0, bucket_cap_mb=0.05, first_bucket_mb=0.01)
    launched = []
    eng._collective = lambda b, view: launched.append(b.index)  # no process group needed
    emb = m.model.embed_tokens
    owners = eng.param_bucket[id(emb)]
    assert eng.num_split_params >= 1 and len(owners) >= 3
    unit = 1024 * world  # fp32: 4 KiB pages per shard
    prev_end = None
    for b in eng.buckets:
        assert b.start % unit == 0 and b.end % unit == 0 and b.end > b.start
        if prev_end is not None and b.start != prev_end:
            assert b.start > prev_end  # only region padding between buckets
        prev_end = b.end
    cap = int(0.05 * 2 ** 20 / 4)
    assert max(b.end - b.start for b in eng.buckets) <= 2 * cap + unit
    # the split parameter's slices are contiguous consecutive buckets covering it exactly
    o = eng.param_offset(emb)
    assert owners[0].start <= o and owners[-1].end >= o + emb.numel()
    assert [b.index for b in owners] == list(range(owners[0].index, owners[-1].index + 1))
    # ready signalling: every bucket launches exactly once, in index order, after its last parameter
    eng.prepare_backward()
    for p in eng.params():
        eng._on_param_ready(p)
    if world > 1:  # (a single rank has nothing to communicate: no signalling)
        assert launched == list(range(len(eng.buckets)))
        assert eng.bucket_pending() == [0] * len(eng.buckets) and all(b.ready for b in eng.buckets)
        with pytest.raises(RuntimeError, match="twice"):
            eng._on_param_ready(emb)


def test_full_smollm3_plan_at_8_ranks_on_meta():
    """SmolLM3-3B full-param shapes at N=8 (meta tensors, registration order of the real model): the 525 MB
    tied embedding is split, no bucket exceeds two caps."""
    from llm_fine_tune_distributed_amd.models import smollm3_3b
    c = smollm3_3b()

    def P(*shape):
        return torch.nn.Parameter(torch.empty(*shape, device="meta", dtype=torch.bfloat16))

    m = torch.nn.Module()
    m.embed_tokens = P(c.vocab_size, c.hidden_size)
    m.layers = torch.nn.ModuleList()
    for _ in range(c.num_hidden_layers):
        layer = torch.nn.Module()
        layer.input_layernorm = P(c.hidden_size)
        layer.qkv_proj = P(c.qkv_size, c.hidden_size)
        layer.o_proj = P(c.hidden_size, c.q_size)
        layer.post_attention_layernorm = P(c.hidden_size)
        layer.gate_up_proj = P(2 * c.intermediate_size, c.hidden_size)
        layer.down_proj = P(c.hidden_size, c.intermediate_size)
        m.layers.append(layer)
    m.norm = P(c.hidden_size)
    eng = DDPEngine(m, world_size=8, rank=0)
    sizes = [(b.end - b.start) * 2 / 2 ** 20 for b in eng.buckets]
    assert 100 < eng.bucket_cap_mb <= 256
    assert eng.num_split_params == 1 and len(eng.param_bucket[id(m.embed_tokens)]) >= 2
    assert max(sizes) <= 2 * eng.bucket_cap_mb + 1
    assert sizes[0] < 50  # the last layer's down_proj alone (a parameter is never split below 2 caps)


def _random_plans():
    import random
    rnd = random.Random(0)
    for case in range(60):
        n = rnd.randint(1, 40)
        sizes = [rnd.choice([1, 7, 64, 1000, 4096, 70000, 300000, 2_000_000]) for _ in range(n)]
        nd = rnd.randint(0, n)
        region = [0] * nd + [1] * (n - nd)
        world = rnd.choice([1, 2, 4, 8])
        pad_unit = 2048 * world
        cap = rnd.choice([pad_unit, 50_000, 400_000])
        first_cap = rnd.choice([pad_unit, 20_000])
        split_at = rnd.choice([0, 2 * cap])
        tied = rnd.choice([-1, rnd.randrange(n)])
        yield sizes, region, tied, 64, pad_unit, cap, first_cap, split_at


def test_native_bucket_planner_matches_python_twin():
    """csrc/ddp_reducer.cpp ddp_plan == the Python twin on random parameter lists (regions, oversized splits, tied
    weight in buckets of its own, world sizes 1-8)."""
    from llm_fine_tune_distributed_amd.ops import _ext
    from llm_fine_tune_distributed_amd.parallel.ddp import _plan_python
    assert _ext.load(), _ext.load_error()
    for args in _random_plans():
        assert list(_ext.ops().ddp_plan(*args)) == _plan_python(*args), args


def test_native_ready_tracker_matches_python_twin():
    """Launch order, pending counts and the double-signal error of the native tracker vs the Python twin."""
    import random
    from llm_fine_tune_distributed_amd.parallel.ddp import ReadyTracker, _plan_python
    rnd = random.Random(1)
    for args in list(_random_plans())[:20]:
        plan = _plan_python(*args)
        nb, np_ = plan[1], plan[2]
        k = 4 + np_ + 3 * nb
        ptr = plan[k:k + np_ + 1]
        own = plan[k + np_ + 1:k + np_ + 1 + ptr[-1]]
        nat, py = ReadyTracker(ptr, own, nb, native=True), ReadyTracker(ptr, own, nb, native=False)
        assert nat.native and not py.native
        for _ in range(2):  # reset between backwards
            nat.reset(), py.reset()
            order = list(range(np_))
            rnd.shuffle(order)
            cut = rnd.randint(0, np_)
            for i in order[:cut]:
                assert nat.mark(i) == py.mark(i)
                assert nat.pending() == py.pending()
            assert nat.drain() == py.drain()
        if np_:
            nat.reset(), py.reset()
            assert nat.mark(order[0]) == py.mark(order[0])
            with pytest.raises(RuntimeError, match="twice"):
                nat.mark(order[0])
            with pytest.raises(RuntimeError, match="twice"):
                py.mark(order[0])


def test_engine_uses_native_reducer():
    m = build_model(tiny(), dtype=torch.float32, seed=0)
    eng = DDPEngine(m, world_size=2, rank=0, bucket_cap_mb=0.05, first_bucket_mb=0.01)
    assert eng._tracker.native


def test_fit_link_recovers_alpha_and_bandwidth():
    from llm_fine_tune_distributed_amd.parallel.ddp import fit_link
    for world, alpha_us, gbps in ((2, 25.0, 80.0), (8, 60.0, 140.0), (4, 5.0, 40.0)):
        pts = [(b, alpha_us * 1e-6 + b / (world * gbps * 1e9)) for b in (4 << 20, 16 << 20, 32 << 20)]
        a, l = fit_link(pts, world)
        assert a == pytest.approx(alpha_us, rel=1e-6) and l == pytest.approx(gbps, rel=1e-6)
    with pytest.raises(ValueError):
        fit_link([(1 << 20, 1e-4)], 2)
    # a noisy probe whose larger message was no slower (slope <= 0) clamps L to 1000 GB/s; strict -> None (the
    # trainer then keeps the modelled plan) instead of a 256 MB bucket cap
    noisy = [(4 << 20, 3e-4), (32 << 20, 2.9e-4)]
    assert fit_link(noisy, 8)[1] == 1000.0
    assert fit_link(noisy, 8, strict=True) is None
    good = [(b, 30e-6 + b / (8 * 100e9)) for b in (4 << 20, 32 << 20)]
    assert fit_link(good, 8, strict=True) == pytest.approx(fit_link(good, 8))


def test_bucket_plan_follows_the_measured_link():
    """The injected probe result (alpha, L) moves the bucket cap: a slower per-call latency or a faster link asks
    for larger buckets (latency share <= ~15 %), the modelled defaults are used only without a probe."""
    from llm_fine_tune_distributed_amd.models import smollm3_3b
    c = smollm3_3b()
    m = torch.nn.Module()  # SmolLM3-3B parameter shapes on the meta device (no 6 GB allocation)
    m.embed_tokens = torch.nn.Parameter(torch.empty(c.vocab_size, c.hidden_size, device="meta", dtype=torch.bfloat16))
    m.layers = torch.nn.ParameterList([torch.nn.Parameter(torch.empty(2 * c.intermediate_size, c.hidden_size,
                                                                      device="meta", dtype=torch.bfloat16))
                                       for _ in range(c.num_hidden_layers)])
    caps = {}
    for name, link in (("model", None), ("slow_call", (120.0, 100.0)), ("fast_call", (8.0, 100.0)),
                       ("fast_link", (30.0, 300.0))):
        eng = DDPEngine(m, world_size=4, rank=0, link=link)
        assert eng.plan_source == ("model" if link is None else "probe")
        caps[name] = eng.bucket_cap_mb
        if link is not None:
            assert caps[name] == plan_bucket_mb(4, alpha_us=link[0], link_gbps=link[1],
                                                total_bytes=sum(p.numel() for p in m.parameters()) * 2)
    assert caps["slow_call"] > caps["model"] > caps["fast_call"]
    assert caps["fast_link"] > caps["model"]
    assert DDPEngine(m, world_size=4, rank=0, bucket_cap_mb=20.0, link=(120.0, 100.0)).plan_source == "user"


def _probe_rank(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llm_fine_tune_distributed_amd.parallel.ddp import fit_link, measure_link
    pts = measure_link(world, torch.device("cpu"), sizes_mb=(0.25, 2.0), iters=2)
    torch.save({"pts": pts, "fit": fit_link(pts, world)}, f"{out}/p{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_measure_link_is_identical_on_every_rank(world, tmp_path):
    """The startup probe takes the max over ranks, so every rank fits the same alpha / L and builds the same plan."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_probe_rank, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"p{r}.pt") for r in range(world)]
    assert len(res[0]["pts"]) == 2 and res[0]["pts"][1][0] > res[0]["pts"][0][0]
    for r in res[1:]:
        assert r["pts"] == res[0]["pts"] and r["fit"] == res[0]["fit"]
    assert res[0]["fit"][0] >= 1.0 and 1.0 <= res[0]["fit"][1] <= 1000.0
