"""Trainer-level GPU checks: optimizer/forward overlap gives the same training trajectory as the
serial update; packed and padded batches agree on GPU."""
import pytest
import torch

from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer

pytestmark = pytest.mark.gpu


def _cfg():
    return tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                intermediate_size=512, vocab_size=1024, num_hidden_layers=3)


def _run(overlap, packing=False, steps=4, padding_free=None, **kw):
    cfg = _cfg()
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=0)
    ds = TokenizedDataset.synthetic(64, cfg.vocab_size, 30, 90, seed=2)
    a = SFTConfig(output_dir="/tmp/sftamd_t", per_device_train_batch_size=4, max_steps=steps, learning_rate=1e-3,
                  logging_steps=1, jsonl_log=False, save_strategy="no", optimizer_overlap=overlap, packing=packing,
                  dataloader_drop_last=True, padding_free=padding_free, **kw)
    t = SFTTrainer(model=m, args=a, train_dataset=ds)
    t.train()
    return [h["loss"] for h in t.state.log_history if "loss" in h], t.engine.param_flat.float().clone()


def test_overlap_matches_serial_update():
    l0, p0 = _run(False)
    l1, p1 = _run(True)
    assert l0 == pytest.approx(l1, rel=1e-6, abs=1e-6)
    assert torch.equal(p0, p1)


def test_packing_trains_on_gpu():
    l, p = _run(True, packing=True)
    assert all(torch.isfinite(torch.tensor(l)))


def test_padding_free_default_matches_padded_on_gpu():
    """The GPU default (padding_free) trains like the padded batches: same loss trajectory within bf16 tolerance
    (different M, so different GEMM tilings), finite, and the trainer reports the flattened mode."""
    l_pad, p_pad = _run(True, padding_free=False)
    l_pf, p_pf = _run(True)
    assert l_pf == pytest.approx(l_pad, rel=2e-2)
    assert ((p_pf - p_pad).norm() / p_pad.norm()).item() < 1e-2


@pytest.mark.parametrize("shard", [False, True])
def test_lora_overlap_matches_serial_update(shard):
    """LoRA refreshes every layer's wide weight (B blocks, A rows) in ONE batched copy at the first forward after an
    update: with the update overlapped on a side stream that copy must still see the finished update of EVERY layer,
    not only of the layers whose forward pre-hooks have run (FlatAdamW and ZeRO-1's ShardedAdamW)."""
    kw = dict(freeze_policy="lora", lora_r=16, lora_alpha=32.0, lora_dropout=0.0, shard_optimizer_state=shard)
    l0, p0 = _run(False, steps=4, **kw)
    l1, p1 = _run(True, steps=4, **kw)
    assert l0 == pytest.approx(l1, rel=1e-6, abs=1e-6)
    assert torch.equal(p0, p1)
