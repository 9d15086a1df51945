"""Multi-process DDP on CPU (gloo, world_size 2): DDP(N) == single process on the same global batch,
ranks stay bit-identical, GA/no_sync semantics and the token-count normalisation hold."""
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


def _flat_state(osd, k):
    """Per-parameter optimizer state (checkpoint format v2) flattened in name order."""
    return torch.cat([v[k].reshape(-1).float() for _, v in sorted(osd["param_state"].items())])


def _run(rank, world, port, out_dir, per_dev, ga, steps, shard=False, tag="", avg_tokens=True, fixed_len=False,
         merge=0, max_len=1024):
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
    ds = TokenizedDataset.synthetic(64, cfg.vocab_size, 12 if fixed_len else 5, 12 if fixed_len else 20, seed=7)
    args = SFTConfig(output_dir=out_dir, per_device_train_batch_size=per_dev, gradient_accumulation_steps=ga,
                     learning_rate=1e-3, max_steps=steps, logging_steps=1, dataloader_drop_last=True,
                     jsonl_log=False, ddp_check_sync_every=1, ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01,
                     save_strategy="no", shard_optimizer_state=shard, average_tokens_across_devices=avg_tokens,
                     ga_merge_max_tokens=merge, max_length=max_len)
    t = SFTTrainer(model=m, args=args, train_dataset=ds)
    out = t.train()
    osd = t.optimizer.state_dict(dst=None)  # full state on every rank (collective in ZeRO-1 mode)
    osd0 = t.optimizer.state_dict(dst=0)  # the checkpoint form: built on rank 0 only
    dst0 = {"empty": not osd0, "host_bytes": t.optimizer.last_state_dict_host_bytes,
            "equal": bool(osd0) and all(torch.equal(_flat_state(osd0, k), _flat_state(osd, k))
                                         for k in ("exp_avg", "exp_avg_sq"))}
    torch.save({"params": t.engine.params_by_name().clone(), "loss": out.training_loss,
                "log": [h for h in t.state.log_history if "loss" in h], "exp_avg": _flat_state(osd, "exp_avg"),
                "exp_avg_sq": _flat_state(osd, "exp_avg_sq"), "sharded": type(t.optimizer).__name__,
                "tied_sparse": t.engine.tied_sparse, "sparse_exchanges": t.engine.sparse_exchanges,
                "replicated_buckets": sum(b.replicated for b in t.engine.buckets), "dst0": dst0,
                "sparse_cap": t.engine.sparse_cap},
               os.path.join(out_dir, f"r{world}_{rank}{tag}.pt"))
    pgm.cleanup_distributed()


def _launch(world, per_dev, ga, steps, d, shard=False, tag="", avg_tokens=True, fixed_len=False, merge=0, max_len=1024):
    port = _free_port()
    if world == 1:
        _run(0, 1, port, d, per_dev, ga, steps, shard, tag, avg_tokens, fixed_len, merge, max_len)
    else:
        mp.spawn(_run, args=(world, port, d, per_dev, ga, steps, shard, tag, avg_tokens, fixed_len, merge, max_len),
                 nprocs=world, join=True)


def test_ddp2_matches_single_process():
    d = tempfile.mkdtemp()
    _launch(1, 4, 1, 3, d)
    _launch(2, 2, 1, 3, d)
    single = torch.load(os.path.join(d, "r1_0.pt"))
    r0 = torch.load(os.path.join(d, "r2_0.pt"))
    r1 = torch.load(os.path.join(d, "r2_1.pt"))
    assert torch.equal(r0["params"], r1["params"])  # ranks bit-identical
    assert torch.allclose(r0["params"], single["params"], atol=1e-5, rtol=1e-4)
    for a, b in zip(single["log"], r0["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-4
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-3


def test_grad_accumulation_equals_big_batch():
    """GA=2 x micro 2 == one micro-batch of 4 (same samples; loss normalised by the step's token count)."""
    d = tempfile.mkdtemp()
    _launch(1, 4, 1, 2, d)
    big = torch.load(os.path.join(d, "r1_0.pt"))
    d2 = tempfile.mkdtemp()
    _launch(1, 2, 2, 2, d2)  # GA run as two passes (ga_merge_max_tokens=0)
    ga = torch.load(os.path.join(d2, "r1_0.pt"))
    assert torch.allclose(ga["params"], big["params"], atol=1e-5, rtol=1e-4)
    for a, b in zip(big["log"], ga["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-5
    d3 = tempfile.mkdtemp()
    _launch(1, 2, 2, 2, d3, merge=4096)  # GA micro-batches merged into one pass (the MI355X default)
    mg = torch.load(os.path.join(d3, "r1_0.pt"))
    assert torch.allclose(mg["params"], big["params"], atol=1e-5, rtol=1e-4)
    for a, b in zip(big["log"], mg["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-5
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-4 * max(1.0, a["grad_norm"])


def test_zero1_sharded_optimizer_matches_replicated():
    """ZeRO-1 (reduce-scatter grads, update 1/world of the params per rank, all-gather them back) gives
    the same parameters, losses, grad norms and (gathered) Adam state as replicated DDP."""
    d = tempfile.mkdtemp()
    _launch(2, 2, 2, 3, d)
    _launch(2, 2, 2, 3, d, shard=True, tag="_z")
    rep = [torch.load(os.path.join(d, f"r2_{r}.pt")) for r in range(2)]
    z = [torch.load(os.path.join(d, f"r2_{r}_z.pt")) for r in range(2)]
    assert z[0]["sharded"] == "ShardedAdamW" and rep[0]["sharded"] == "FlatAdamW"
    assert torch.equal(z[0]["params"], z[1]["params"])  # all-gathered: ranks identical
    assert torch.allclose(z[0]["params"], rep[0]["params"], atol=1e-6, rtol=1e-5)
    for k in ("exp_avg", "exp_avg_sq"):
        assert torch.allclose(z[0][k], rep[0][k], atol=1e-7, rtol=1e-4)
    for a, b in zip(rep[0]["log"], z[0]["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-5
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-4 * max(1.0, a["grad_norm"])


def test_zero1_world4_matches_replicated():
    """ZeRO-1 at world_size 4 (bucket shards of uneven sizes, first-bucket split, 4-way reduce-scatter /
    all-gather) against replicated DDP at the same world size: the code path bench.py takes at N = 4 / 8."""
    d = tempfile.mkdtemp()
    _launch(4, 1, 2, 2, d)
    _launch(4, 1, 2, 2, d, shard=True, tag="_z")
    rep = [torch.load(os.path.join(d, f"r4_{r}.pt")) for r in range(4)]
    z = [torch.load(os.path.join(d, f"r4_{r}_z.pt")) for r in range(4)]
    assert z[0]["sharded"] == "ShardedAdamW"
    for r in range(1, 4):
        assert torch.equal(z[0]["params"], z[r]["params"])
        assert torch.equal(rep[0]["params"], rep[r]["params"])
    assert torch.allclose(z[0]["params"], rep[0]["params"], atol=1e-6, rtol=1e-5)
    for k in ("exp_avg", "exp_avg_sq"):
        assert torch.allclose(z[0][k], rep[0][k], atol=1e-7, rtol=1e-4)
    for a, b in zip(rep[0]["log"], z[0]["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-5


def test_local_token_normalisation_matches_single_process():
    """average_tokens_across_devices=False (HF: each rank's loss is its LOCAL mean, DDP averages the
    gradients): with equal token counts per rank, world 2 == world 1 on the same global batch — the
    SUM-reduced buckets must not make the gradients world_size times larger."""
    d = tempfile.mkdtemp()
    _launch(1, 4, 1, 2, d, tag="_l", avg_tokens=False, fixed_len=True)
    _launch(2, 2, 1, 2, d, tag="_l", avg_tokens=False, fixed_len=True)
    single = torch.load(os.path.join(d, "r1_0_l.pt"))
    r0 = torch.load(os.path.join(d, "r2_0_l.pt"))
    assert torch.allclose(r0["params"], single["params"], atol=1e-5, rtol=1e-4)
    for a, b in zip(single["log"], r0["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-4
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-3 * max(1.0, a["grad_norm"])


def _save_zero_ckpt(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import llm_fine_tune_distributed_amd.parallel.process_group as pgm
    pgm._STATE = None
    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
    cfg = tiny()
    m = build_model(cfg, dtype=torch.float32, seed=3)
    ds = TokenizedDataset.synthetic(64, cfg.vocab_size, 5, 20, seed=7)
    args = SFTConfig(output_dir=out_dir, per_device_train_batch_size=2, learning_rate=1e-3, max_steps=2,
                     logging_steps=0, jsonl_log=False, save_strategy="steps", save_steps=2,
                     shard_optimizer_state=True, ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01,
                     master_weights=True)
    SFTTrainer(model=m, args=args, train_dataset=ds).train()
    pgm.cleanup_distributed()


def test_zero1_checkpoint_resumes_at_another_world_size():
    """The optimizer checkpoint is keyed by parameter name, not by the world-size-dependent flat layout:
    a ZeRO-1 checkpoint written at world 4 loads into a replicated optimizer at world 1 exactly."""
    d = tempfile.mkdtemp()
    mp.spawn(_save_zero_ckpt, args=(4, _free_port(), d), nprocs=4, join=True)
    path = os.path.join(d, "checkpoint-2")
    saved = torch.load(os.path.join(path, "optimizer.pt"), weights_only=True)
    assert saved["format"] == "sftamd-adamw-v2" and saved["saved_world_size"] == 4
    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
    from llm_fine_tune_distributed_amd.train import checkpoint as ck
    import llm_fine_tune_distributed_amd.parallel.process_group as pgm
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    pgm._STATE = None
    cfg = tiny()
    t = SFTTrainer(model=build_model(cfg, dtype=torch.float32, seed=5),
                   args=SFTConfig(output_dir=tempfile.mkdtemp(), jsonl_log=False, max_steps=1, master_weights=True),
                   train_dataset=TokenizedDataset.synthetic(8, cfg.vocab_size, 5, 20, seed=7))
    from llm_fine_tune_distributed_amd.train.optim import LRScheduler, get_schedule
    t.scheduler = LRScheduler(t.optimizer, get_schedule("linear", 10))
    ck.load_checkpoint(path, t.model, t.optimizer, t.scheduler, 0)
    got = t.optimizer.state_dict()
    assert got["step"] == saved["step"] == 2
    for name, st in saved["param_state"].items():
        for k in ("exp_avg", "exp_avg_sq", "master"):
            assert torch.equal(got["param_state"][name][k], st[k]), (name, k)


@pytest.mark.parametrize("world,shard,ga,merge", [(2, True, 2, 0), (2, False, 1, 0), (4, True, 1, 0),
                                                  (4, False, 2, 32768)])
def test_tied_embedding_sparse_exchange(world, shard, ga, merge, monkeypatch):
    """Sparse tied-embedding gradient (default for world > 1: the lm_head part all-reduced early in buckets of
    its own, the embedding rows all-gathered after backward, the tied weight replicated under ZeRO-1) == the dense
    bucket path, and both == one process on the same global batch; GA no_sync passes keep the dense accumulation."""
    d = tempfile.mkdtemp()
    per_dev = 4 // world if ga == 1 else 2 // (world // 2 if world > 2 else 1)
    per_dev = max(1, per_dev)
    monkeypatch.setenv("SFTAMD_TIED_SPARSE", "1")
    # max_length stays at its default (1024): the gather bound comes from the data the collator will see
    # (samples of 5..20 tokens), not from max_length
    _launch(world, per_dev, ga, 3, d, shard=shard, tag="_sp", merge=merge)
    monkeypatch.setenv("SFTAMD_TIED_SPARSE", "0")
    _launch(world, per_dev, ga, 3, d, shard=shard, tag="_dn", merge=merge)
    sp = [torch.load(os.path.join(d, f"r{world}_{r}_sp.pt")) for r in range(world)]
    dn = torch.load(os.path.join(d, f"r{world}_0_dn.pt"))
    assert sp[0]["tied_sparse"] and sp[0]["sparse_exchanges"] == 3 and sp[0]["replicated_buckets"] >= 1
    # a host-known gather size (no device sync) unless the bound is too large for the vocabulary (merged GA passes)
    assert (sp[0]["sparse_cap"] > 0) == (merge == 0), sp[0]["sparse_cap"]
    if merge == 0:
        assert sp[0]["sparse_cap"] <= per_dev * 20, sp[0]["sparse_cap"]
    assert not dn["tied_sparse"] and dn["sparse_exchanges"] == 0 and dn["replicated_buckets"] == 0
    for r in range(1, world):
        assert torch.equal(sp[0]["params"], sp[r]["params"])  # replicated tied weight stays bit-identical
    assert torch.allclose(sp[0]["params"], dn["params"], atol=1e-5, rtol=1e-4)
    assert torch.allclose(sp[0]["exp_avg_sq"], dn["exp_avg_sq"], atol=1e-8, rtol=1e-3)
    for a, b in zip(dn["log"], sp[0]["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-4
        assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-3 * max(1.0, a["grad_norm"])


@pytest.mark.parametrize("world", [2, 4])
def test_zero1_state_dict_gathers_to_rank0_only(world):
    """Checkpoint form of the ZeRO-1 optimizer state: rank 0 receives every shard (equal to the all-gathered state);
    the other ranks return nothing and copy nothing to the host (O(shard) memory)."""
    d = tempfile.mkdtemp()
    _launch(world, 1, 1, 2, d, shard=True, tag="_g")
    recs = [torch.load(os.path.join(d, f"r{world}_{r}_g.pt")) for r in range(world)]
    assert recs[0]["sharded"] == "ShardedAdamW"
    assert not recs[0]["dst0"]["empty"] and recs[0]["dst0"]["equal"] and recs[0]["dst0"]["host_bytes"] > 0
    for r in recs[1:]:
        assert r["dst0"]["empty"] and r["dst0"]["host_bytes"] == 0
