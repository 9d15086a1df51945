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


def _run(rank, world, port, out_dir, per_dev, ga, steps):
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
    ds = TokenizedDataset.synthetic(64, cfg.vocab_size, 5, 20, seed=7)
    args = SFTConfig(output_dir=out_dir, per_device_train_batch_size=per_dev, gradient_accumulation_steps=ga,
                     learning_rate=1e-3, max_steps=steps, logging_steps=1, dataloader_drop_last=True,
                     jsonl_log=False, ddp_check_sync_every=1, ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01,
                     save_strategy="no")
    t = SFTTrainer(model=m, args=args, train_dataset=ds)
    out = t.train()
    torch.save({"params": t.engine.param_flat.clone(), "loss": out.training_loss,
                "log": [h for h in t.state.log_history if "loss" in h]},
               os.path.join(out_dir, f"r{world}_{rank}.pt"))
    pgm.cleanup_distributed()


def _launch(world, per_dev, ga, steps, d):
    port = _free_port()
    if world == 1:
        _run(0, 1, port, d, per_dev, ga, steps)
    else:
        mp.spawn(_run, args=(world, port, d, per_dev, ga, steps), nprocs=world, join=True)


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
    _launch(1, 2, 2, 2, d2)
    ga = torch.load(os.path.join(d2, "r1_0.pt"))
    assert torch.allclose(ga["params"], big["params"], atol=1e-5, rtol=1e-4)
    for a, b in zip(big["log"], ga["log"]):
        assert abs(a["loss"] - b["loss"]) < 1e-5
