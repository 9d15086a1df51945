"""Context parallelism (ring attention) on CPU / gloo: world 2 and 4 against single-process attention and a
single-process model step on the full sequences."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _chunk_rows(B, T, L, r, layout="contiguous", world=1):
    if layout == "zigzag":
        h = L // 2
        return torch.cat([torch.cat([torch.arange(b * T + r * h, b * T + (r + 1) * h),
                                     torch.arange(b * T + (2 * world - 1 - r) * h, b * T + (2 * world - r) * h)])
                          for b in range(B)])
    return torch.cat([torch.arange(b * T + r * L, b * T + (r + 1) * L) for b in range(B)])


def _op_worker(rank, world, port, out_dir, layout):
    dist = _init(rank, world, port)
    from llm_fine_tune_distributed_amd.ops import reference as ref
    from llm_fine_tune_distributed_amd.parallel.context_parallel import ring_attention
    torch.manual_seed(0)
    B, L, nq, nkv, D = 2, 6, 4, 2, 16
    T = L * world
    qkv = torch.randn(B * T, (nq + 2 * nkv) * D)
    dout = torch.randn(B * T, nq * D)
    cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32)
    full = qkv.clone().requires_grad_(True)
    o_ref = ref.attention(full, nq, nkv, D, cu, None, True)
    (g_ref,) = torch.autograd.grad(o_ref, full, dout)
    rows = _chunk_rows(B, T, L, rank, layout, world)
    loc = qkv[rows].clone().requires_grad_(True)
    cu_l = torch.arange(0, (B + 1) * L, L, dtype=torch.int32)
    o = ring_attention(loc, cu_l, L, nq, nkv, D, dist.group.WORLD, layout=layout)
    (g,) = torch.autograd.grad(o, loc, dout[rows])
    torch.save({"eo": (o - o_ref[rows]).abs().max().item(), "eg": (g - g_ref[rows]).abs().max().item(),
                "gn": g_ref[rows].abs().max().item()}, os.path.join(out_dir, f"op{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("layout", ["zigzag", "contiguous"])
@pytest.mark.parametrize("world", [2, 4])
def test_ring_attention_matches_full_attention(world, layout):
    d = tempfile.mkdtemp()
    mp.spawn(_op_worker, args=(world, _free_port(), d, layout), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(os.path.join(d, f"op{r}.pt"))
        assert res["eo"] < 1e-5, res
        assert res["eg"] < 1e-5 * max(1.0, res["gn"]), res


def _model_worker(rank, world, port, out_dir, layout):
    dist = _init(rank, world, port)
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.parallel.context_parallel import shard_batch
    torch.manual_seed(0)
    cfg = tiny("smollm3", num_hidden_layers=4)
    B, T = 2, 21  # T not a multiple of world: exercises the padding of the last chunk
    ids = torch.randint(0, cfg.vocab_size, (B, T))
    labels = ids.clone()
    labels[1, 15:] = -100
    m = build_model(cfg, dtype=torch.float32, seed=7)
    m.enable_context_parallel(dist.group.WORLD, layout)
    b = shard_batch({"input_ids": ids, "labels": labels}, rank, world, layout=layout)
    n = torch.tensor([float(b["num_items"])])
    dist.all_reduce(n)
    m.reset_grad_use_counters()
    out = m(b["input_ids"], labels=b["labels"], position_ids=b["position_ids"], shift_labels=False,
            num_items_in_batch=n)
    out.loss.backward()
    loss = out.loss.detach().clone()
    dist.all_reduce(loss)
    grads = {}
    for name, p in m.named_parameters():
        g = p.grad if p.grad is not None else getattr(p, "main_grad", None)
        g = torch.zeros_like(p) if g is None else g.clone()
        dist.all_reduce(g)
        grads[name] = g
    torch.save({"loss": loss.item(), "grads": grads, "n": n.item()}, os.path.join(out_dir, f"m{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("layout", ["zigzag", "contiguous"])
@pytest.mark.parametrize("world", [2, 4])
def test_context_parallel_model_matches_single_process(world, layout):
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    d = tempfile.mkdtemp()
    mp.spawn(_model_worker, args=(world, _free_port(), d, layout), nprocs=world, join=True)
    torch.manual_seed(0)
    cfg = tiny("smollm3", num_hidden_layers=4)
    B, T = 2, 21
    ids = torch.randint(0, cfg.vocab_size, (B, T))
    labels = ids.clone()
    labels[1, 15:] = -100
    m = build_model(cfg, dtype=torch.float32, seed=7)
    n = float((labels[:, 1:] != -100).sum())
    m.reset_grad_use_counters()
    out = m(ids, labels=labels, num_items_in_batch=torch.tensor([n]))
    out.loss.backward()
    r0 = torch.load(os.path.join(d, "m0.pt"))
    assert r0["n"] == n
    assert abs(r0["loss"] - out.loss.item()) < 1e-5
    for name, p in m.named_parameters():
        g = p.grad if p.grad is not None else getattr(p, "main_grad", None)
        e = (r0["grads"][name] - g).abs().max().item()
        assert e < 1e-5 * max(1.0, g.abs().max().item()), (name, e)


def _trainer_worker(rank, world, port, out_dir, cp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import llm_fine_tune_distributed_amd.parallel.process_group as pgm
    pgm._STATE = None
    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
    torch.manual_seed(0)
    cfg = tiny()
    m = build_model(cfg, dtype=torch.float32, seed=3)
    ds = TokenizedDataset.synthetic(32, cfg.vocab_size, 9, 23, seed=7)
    args = SFTConfig(output_dir=out_dir, per_device_train_batch_size=4, gradient_accumulation_steps=2,
                     learning_rate=1e-3, max_steps=2, logging_steps=1, dataloader_drop_last=True, jsonl_log=False,
                     save_strategy="no", context_parallel_size=cp, ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01)
    t = SFTTrainer(model=m, args=args, train_dataset=ds)
    t.train()
    torch.save({"params": t.engine.params_by_name().clone(), "log": [h for h in t.state.log_history if "loss" in h]},
               os.path.join(out_dir, f"t{world}_{cp}_{rank}.pt"))
    pgm.cleanup_distributed()


def test_trainer_context_parallel_equals_single_process():
    """SFTTrainer with context_parallel_size = 2 on 2 ranks (one CP group, dp 1) trains exactly like one
    process on the same batches: same losses, grad norms and parameters."""
    d = tempfile.mkdtemp()
    _trainer_worker(0, 1, _free_port(), d, 1)
    mp.spawn(_trainer_worker, args=(2, _free_port(), d, 2), nprocs=2, join=True)
    single = torch.load(os.path.join(d, "t1_1_0.pt"))
    cp = [torch.load(os.path.join(d, f"t2_2_{r}.pt")) for r in range(2)]
    assert torch.equal(cp[0]["params"], cp[1]["params"])
    # Adam normalises each gradient element: where a gradient is ~0 its update is sign-sensitive to the
    # last-bit differences of the blockwise attention, so compare the bulk tightly and bound the rest by lr
    diff = (cp[0]["params"] - single["params"]).abs()
    assert diff.max().item() <= 2 * 2e-3 + 1e-6, diff.max().item()  # two steps of at most ~lr each
    assert (diff > 1e-5).float().mean().item() < 1e-3, (diff > 1e-5).float().mean().item()
    for a, b in zip(single["log"], cp[0]["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-4 * max(1.0, abs(a["loss"])), (a, b)
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-4 * max(1.0, a["grad_norm"]), (a, b)


def test_zigzag_balances_causal_work():
    """Every rank computes the same number of half-chunk blocks at every ring step (contiguous: 0 .. 1)."""
    from llm_fine_tune_distributed_amd.parallel.context_parallel import _zz_pairs
    for n in (2, 4, 8):
        for s in range(n):
            work = [sum(0.5 if c else 1.0 for _, _, c in _zz_pairs(r, (r - s) % n, n)) for r in range(n)]
            assert work == [2.0] * n, (n, s, work)  # two (L/2)^2 blocks per rank per step
