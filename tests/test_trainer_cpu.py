"""Trainer semantics on CPU: BASELINE config #1 (8 synthetic Q&A pairs, 1 optimizer step),
artifacts, checkpoint/resume, LoRA, LR schedules, callbacks."""
import json
import math
import os

import pytest
import torch

from llm_fine_tune_distributed_amd.data.synthetic import generate_qa
from llm_fine_tune_distributed_amd.data.tokenizer import load_tokenizer
from llm_fine_tune_distributed_amd.models import build_model, tiny
from llm_fine_tune_distributed_amd.train import (PerplexityCallback, SFTConfig, SFTTrainer, TrainingHistoryCallback)
from llm_fine_tune_distributed_amd.train import checkpoint as ckpt
from llm_fine_tune_distributed_amd.train.optim import get_schedule


@pytest.fixture(scope="module")
def tk():
    return load_tokenizer()


def _model(seed=0):
    return build_model(tiny(vocab_size=1024), dtype=torch.float32, seed=seed)


def test_baseline_config1_one_step(tmp_path, tk):
    """8 synthetic Q&A pairs, 1 optimizer step, reference SFTConfig kwargs verbatim (training.py:258-287)."""
    rows = generate_qa(8, seed=0)
    args = SFTConfig(output_dir=str(tmp_path / "checkpoints"), per_device_train_batch_size=8,
                     per_device_eval_batch_size=8, gradient_accumulation_steps=1, learning_rate=5e-5,
                     max_grad_norm=1.0, num_train_epochs=1, logging_steps=2, logging_first_step=True, save_steps=500,
                     bf16=True, eval_strategy="steps", eval_steps=10, save_strategy="steps",
                     load_best_model_at_end=True, metric_for_best_model="eval_loss", greater_is_better=False,
                     save_total_limit=3, dataloader_pin_memory=True, dataloader_num_workers=0,
                     remove_unused_columns=False, gradient_checkpointing=True, dataloader_drop_last=True,
                     max_seq_length=1024, packing=False, ddp_backend=None)
    h = TrainingHistoryCallback()
    t = SFTTrainer(model=_model(), args=args, train_dataset=rows, eval_dataset=rows[:4], processing_class=tk,
                   callbacks=[h, PerplexityCallback()])
    before = t.engine.param_flat.clone()
    out = t.train()
    assert out.global_step == 1
    assert not torch.equal(before, t.engine.param_flat)
    first = h.history[0]
    assert {"loss", "grad_norm", "learning_rate", "epoch", "perplexity"} <= set(first)
    assert math.isclose(first["perplexity"], math.exp(first["loss"]), rel_tol=1e-6)
    assert {"train_runtime", "train_samples_per_second", "train_loss"} <= set(h.history[-1])


def test_save_model_hf_layout_roundtrip(tmp_path, tk):
    m = _model()
    t = SFTTrainer(model=m, args=SFTConfig(output_dir=str(tmp_path), jsonl_log=False), train_dataset=generate_qa(4),
                   processing_class=tk)
    t.save_model(str(tmp_path / "best_model"))
    files = set(os.listdir(tmp_path / "best_model"))
    assert {"model.safetensors", "config.json", "generation_config.json", "tokenizer.json"} <= files
    from safetensors.torch import load_file
    sd = load_file(str(tmp_path / "best_model" / "model.safetensors"))
    assert "lm_head.weight" not in sd and "model.layers.0.self_attn.q_proj.weight" in sd  # tied, HF names
    m2 = ckpt.from_pretrained(str(tmp_path / "best_model"), dtype=torch.float32)
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n


def test_sharded_save(tmp_path):
    m = _model()
    ckpt.save_state_dict_sharded(m.hf_state_dict(), str(tmp_path), max_shard_size=200_000)
    assert os.path.exists(tmp_path / "model.safetensors.index.json")
    sd = ckpt.load_state_dict(str(tmp_path))
    assert set(sd) == set(m.hf_state_dict())


def test_checkpoint_resume_continuity(tmp_path, tk):
    """Train 4 steps straight vs 2 steps + resume 2 steps: identical weights."""
    rows = generate_qa(32, seed=5)

    def mk(out, max_steps, save_steps):
        a = SFTConfig(output_dir=str(out), per_device_train_batch_size=4, gradient_accumulation_steps=1,
                      learning_rate=1e-3, max_steps=max_steps, logging_steps=1, save_steps=save_steps,
                      dataloader_drop_last=True, jsonl_log=False, lr_scheduler_type="cosine", warmup_steps=1)
        return SFTTrainer(model=_model(1), args=a, train_dataset=rows, processing_class=tk)

    t_full = mk(tmp_path / "a", 4, 0)
    t_full.train()
    t1 = mk(tmp_path / "b", 4, 2)
    t1.args.max_steps = 2
    t1.train()
    assert os.path.exists(tmp_path / "b" / "checkpoint-2" / "optimizer.pt")
    t2 = mk(tmp_path / "b", 4, 0)
    out = t2.train(resume_from_checkpoint="auto")
    assert out.global_step == 4
    assert torch.allclose(t2.engine.param_flat, t_full.engine.param_flat, atol=1e-6)


def test_lora_trains_only_adapters(tmp_path, tk):
    a = SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=4, max_steps=2, learning_rate=1e-2,
                  freeze_policy="lora", lora_r=4, jsonl_log=False)
    m = _model()
    base = m.model.layers[0].self_attn.qkv_proj.detach().clone()
    t = SFTTrainer(model=m, args=a, train_dataset=generate_qa(16), processing_class=tk)
    assert t.trainable_params < t.total_params
    t.train()
    assert torch.equal(base, m.model.layers[0].self_attn.qkv_proj)
    B = m.model.layers[0].self_attn.lora["qkv"].B[0]
    assert B.abs().sum() > 0  # adapters moved
    t.save_model(str(tmp_path / "lora_model"))
    assert os.path.exists(tmp_path / "lora_model" / "adapter_model.safetensors")


def test_schedules():
    lin = get_schedule("linear", 10, 0)
    assert lin(0) == 1.0 and lin(5) == 0.5 and lin(10) == 0.0
    cos = get_schedule("cosine", 10, 2)
    assert cos(1) == 0.5 and abs(cos(2) - 1.0) < 1e-9 and abs(cos(10)) < 1e-9
    assert get_schedule("constant", 10)(7) == 1.0


def test_stochastic_rounding_twin_unbiased():
    from llm_fine_tune_distributed_amd.ops import reference as ref
    x = torch.full((1 << 16,), 1.0 + 2 ** -9)  # 1/4 of the way from bf16 1.0 to the next value 1 + 2^-7
    r = ref.bf16_stochastic_round(x, seed=3, offset=11)
    assert set(r.float().unique().tolist()) == {1.0, 1.0 + 2 ** -7}
    assert abs(r.float().mean().item() - (1.0 + 2 ** -9)) < 2e-4
    assert torch.equal(r, ref.bf16_stochastic_round(x, seed=3, offset=11))  # counter-based: reproducible
    assert not torch.equal(r, ref.bf16_stochastic_round(x, seed=4, offset=11))
    y = torch.tensor([float("inf"), -float("inf"), -3.5])
    assert torch.equal(ref.bf16_stochastic_round(y, 1).float(), y)


def test_bf16_optimizer_state_trains(tmp_path, tk):
    """optim_state_dtype="bf16": bf16 params + bf16 moments (stochastic rounding) — torch AdamW's state
    dtype for the reference's bf16 model — trains and tracks the fp32-state run closely."""
    rows = generate_qa(16, seed=2)
    res = {}
    for st in ("fp32", "bf16"):
        a = SFTConfig(output_dir=str(tmp_path / st), per_device_train_batch_size=4, max_steps=3, learning_rate=1e-3,
                      jsonl_log=False, optim_state_dtype=st, logging_steps=1)
        m = build_model(tiny(vocab_size=1024), dtype=torch.bfloat16, seed=0)
        t = SFTTrainer(model=m, args=a, train_dataset=rows, processing_class=tk)
        assert t.optimizer.exp_avg.dtype == (torch.bfloat16 if st == "bf16" else torch.float32)
        out = t.train()
        res[st] = (out.training_loss, t.engine.param_flat.float().clone())
    assert abs(res["fp32"][0] - res["bf16"][0]) < 0.05 * abs(res["fp32"][0])
    d = (res["fp32"][1] - res["bf16"][1]).norm() / res["fp32"][1].norm()
    assert d < 1e-2


def test_auto_state_dtype_follows_master_weights(tmp_path, tk):
    """"auto" moments: bf16 for the bf16 model (torch parity), fp32 once an fp32 master copy is kept (that path
    writes back with round-to-nearest, where a bf16 exp_avg_sq would stall)."""
    for master, want in ((False, torch.bfloat16), (True, torch.float32)):
        a = SFTConfig(output_dir=str(tmp_path / str(master)), per_device_train_batch_size=2, max_steps=1,
                      jsonl_log=False, master_weights=master)
        assert a.optim_state_dtype == "auto"
        t = SFTTrainer(model=build_model(tiny(vocab_size=1024), dtype=torch.bfloat16, seed=0), args=a,
                       train_dataset=generate_qa(4), processing_class=tk)
        assert t.optimizer.exp_avg.dtype == want and t.optimizer.exp_avg_sq.dtype == want
        assert (t.optimizer.master is not None) == master


def test_reference_freeze_policy_counts(tmp_path, tk):
    a = SFTConfig(output_dir=str(tmp_path), freeze_policy="last_n_layers", max_steps=1, jsonl_log=False,
                  per_device_train_batch_size=2)
    m = _model()
    t = SFTTrainer(model=m, args=a, train_dataset=generate_qa(4), processing_class=tk)
    per_layer = sum(p.numel() for p in m.model.layers[0].parameters())
    assert t.trainable_params == 2 * per_layer + m.config.vocab_size * m.config.hidden_size
    frozen0 = m.model.layers[0].self_attn.qkv_proj.detach().clone()
    t.train()
    assert torch.equal(frozen0, m.model.layers[0].self_attn.qkv_proj)


def test_config_file_and_set_overrides(tmp_path):
    from llm_fine_tune_distributed_amd.train import SFTConfig, apply_overrides
    y = tmp_path / "run.yaml"
    y.write_text("sft_config:\n  learning_rate: 3.0e-5\n  max_seq_length: 2048\n  lora_target_modules: [q_proj, v_proj]\n"
                 "  shard_optimizer_state: true\n")
    base = SFTConfig(learning_rate=1e-4, gradient_accumulation_steps=4)
    cfg = apply_overrides(base, str(y), ["gradient_accumulation_steps=2", "bf16=false", "warmup_ratio=0.1",
                                         "eval_steps=none"])
    assert cfg.learning_rate == 3e-5 and cfg.max_length == 2048 and cfg.lora_target_modules == ["q_proj", "v_proj"]
    assert cfg.gradient_accumulation_steps == 2 and cfg.bf16 is False and cfg.warmup_ratio == 0.1
    assert cfg.shard_optimizer_state is True and cfg.eval_steps is None
    assert base.gradient_accumulation_steps == 4  # the base config is not mutated
    j = tmp_path / "run.json"
    j.write_text('{"optim_state_dtype": "bf16"}')
    assert apply_overrides(base, str(j)).optim_state_dtype == "bf16"
    with pytest.raises(KeyError):
        apply_overrides(base, None, ["learning_rat=1"])
    (tmp_path / "bad.yaml").write_text("not_a_field: 1\n")
    with pytest.raises(KeyError):
        apply_overrides(base, str(tmp_path / "bad.yaml"))


@pytest.mark.parametrize("policy,ckpt", [("full", False), ("full", True), ("lora", False), ("last_n_layers", True)])
def test_grad_norm_from_backward_partials(tmp_path, tk, monkeypatch, policy, ckpt):
    """The gradient norm summed bucket by bucket during backward (default) equals the post-backward full
    pass (SFTAMD_NORM_IN_BWD=0), with GA 2, gradient checkpointing and every freeze policy; updates match."""
    rows = generate_qa(16, seed=1)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("SFTAMD_NORM_IN_BWD", flag)
        args = SFTConfig(output_dir=str(tmp_path / flag), per_device_train_batch_size=4, gradient_accumulation_steps=2,
                         learning_rate=1e-3, max_grad_norm=0.5, max_steps=2, logging_steps=1, save_strategy="no",
                         jsonl_log=False, gradient_checkpointing=ckpt, freeze_policy=policy, lora_r=4,
                         ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01, seed=3)
        h = TrainingHistoryCallback()
        t = SFTTrainer(model=_model(seed=2), args=args, train_dataset=rows, processing_class=tk, callbacks=[h])
        assert t.engine.track_norm == (flag == "1")
        t.train()
        res[flag] = ([x["grad_norm"] for x in h.history if "grad_norm" in x], t.engine.param_flat.clone())
    (n1, p1), (n0, p0) = res["1"], res["0"]
    assert len(n1) == 2 and all(a > 0 for a in n1)
    for a, b in zip(n1, n0):
        assert abs(a - b) <= 1e-5 * max(1.0, b), (a, b)
    assert torch.allclose(p1, p0, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("packing", [False, True])
def test_ga_merge_matches_separate_passes(tmp_path, tk, packing):
    """ga_merge_max_tokens: the GA micro-batches of a step run as ONE pass (re-padded / varlen-concatenated)
    with the same loss, grad norm, metrics and update as running them one by one."""
    rows = generate_qa(16, seed=4)
    res = {}
    for merge in (0, 1 << 16):
        args = SFTConfig(output_dir=str(tmp_path / str(merge)), per_device_train_batch_size=4,
                         gradient_accumulation_steps=2, learning_rate=1e-3, max_steps=2, logging_steps=1,
                         save_strategy="no", jsonl_log=False, packing=packing, ga_merge_max_tokens=merge, seed=1)
        h = TrainingHistoryCallback()
        t = SFTTrainer(model=_model(seed=7), args=args, train_dataset=rows, processing_class=tk, callbacks=[h])
        out = t.train()
        logs = [x for x in h.history if "loss" in x]
        res[merge] = (logs, t.engine.param_flat.clone(), out.metrics["train_samples_per_second"] > 0)
    (l0, p0, _), (l1, p1, _) = res[0], res[1 << 16]
    assert torch.allclose(p0, p1, atol=1e-5, rtol=1e-4)
    for a, b in zip(l0, l1):
        for k in ("loss", "grad_norm", "mean_token_accuracy", "entropy", "num_tokens"):
            assert abs(a[k] - b[k]) <= 1e-5 * max(1.0, abs(a[k])), (k, a[k], b[k])


def test_padding_free_matches_padded_batches(tmp_path, tk):
    """padding_free (TRL's name; the GPU default): every padded micro-batch flattened into one varlen sequence with
    per-sample positions — the same losses, grad norms, token metrics and update as the padded batches, with the
    eval metrics too (the whole batch is kept, nothing dropped at the pack boundary)."""
    rows = generate_qa(24, seed=5)
    res = {}
    for pf in (False, True):
        args = SFTConfig(output_dir=str(tmp_path / str(pf)), per_device_train_batch_size=4,
                         per_device_eval_batch_size=8, gradient_accumulation_steps=2, learning_rate=1e-3, max_steps=2,
                         logging_steps=1, eval_strategy="steps", eval_steps=2, save_strategy="no", jsonl_log=False,
                         padding_free=pf, seed=1)
        h = TrainingHistoryCallback()
        t = SFTTrainer(model=_model(seed=3), args=args, train_dataset=rows[:16], eval_dataset=rows[16:],
                       processing_class=tk, callbacks=[h])
        assert t.packed == pf
        t.train()
        res[pf] = ([x for x in h.history if "loss" in x], [x for x in h.history if "eval_loss" in x],
                   t.engine.param_flat.clone())
    (l0, e0, p0), (l1, e1, p1) = res[False], res[True]
    assert torch.allclose(p0, p1, atol=1e-5, rtol=1e-4)
    for a, b in zip(l0, l1):
        for k in ("loss", "grad_norm", "mean_token_accuracy", "entropy", "num_tokens"):
            assert abs(a[k] - b[k]) <= 1e-5 * max(1.0, abs(a[k])), (k, a[k], b[k])
    assert len(e0) == len(e1) == 1
    for k in ("eval_loss", "eval_mean_token_accuracy", "eval_num_tokens"):
        assert abs(e0[0][k] - e1[0][k]) <= 1e-5 * max(1.0, abs(e0[0][k])), k


@pytest.mark.parametrize("stop", [False, True])
def test_nonfinite_loss_is_reported_at_the_log_cadence(tmp_path, tk, stop):
    """A NaN parameter makes the logged loss non-finite: the trainer records the step (state.nonfinite_loss_steps),
    beats phase "nonfinite_loss" and, with stop_on_nonfinite_loss, stops at that step."""
    rows = generate_qa(16, seed=0)
    args = SFTConfig(output_dir=str(tmp_path / "o"), per_device_train_batch_size=2, gradient_accumulation_steps=1,
                     max_steps=4, logging_steps=1, save_strategy="no", eval_strategy="no", jsonl_log=False,
                     dataset_cache=False, stop_on_nonfinite_loss=stop)
    m = _model()
    t = SFTTrainer(model=m, args=args, train_dataset=rows, processing_class=tk)
    with torch.no_grad():
        t.engine.param_flat.view(-1)[0] = float("nan")
    seen = []
    orig = t.heartbeat.beat
    t.heartbeat.beat = lambda step=None, phase="", **kw: (seen.append(phase), orig(step, phase, **kw))
    out = t.train()
    assert t.state.nonfinite_loss_steps[:1] == [1]
    assert "nonfinite_loss" in seen
    assert out.global_step == (1 if stop else 4)
