"""End-to-end training CLI (the reference's ``python training.py`` flow) on CPU: env contract, config file +
--set overrides, synthetic Q&A data, tiny model, artifacts with the reference's schema."""
import json
import os

import pytest


def test_train_cli_end_to_end(tmp_path, monkeypatch):
    from llm_fine_tune_distributed_amd.cli import train as cli
    out = tmp_path / "out"
    monkeypatch.setenv("OUTPUT_DIR", str(out))
    monkeypatch.setenv("EPOCHS", "1")
    monkeypatch.setenv("BATCH_SIZE", "4")
    monkeypatch.setenv("LEARNING_RATE", "1e-3")
    monkeypatch.setenv("AIM_REPO", str(tmp_path / "aim"))
    from llm_fine_tune_distributed_amd.utils import telemetry
    monkeypatch.setattr(telemetry, "gpu_stats", lambda: [{"index": 0, "gfx_util": 97.0, "power_w": 812.0}])
    cfgf = tmp_path / "run.yaml"
    cfgf.write_text("sft_config:\n  eval_steps: 1\n  logging_steps: 1\n  max_length: 256\n")
    cli.main(["--model", "tiny", "--dataset", "synthetic", "--max-steps", "2", "--max-train-samples", "48",
              "--grad-accum", "2", "--no-gradient-checkpointing", "--config", str(cfgf),
              "--set", "warmup_steps=1", "--set", "lr_scheduler_type=cosine", "--log-step-phases",
              "--log-system-metrics-every", "1"])
    summary = json.load(open(out / "training_summary.json"))
    ref_keys = {"model_name", "dataset_path", "epochs", "batch_size", "learning_rate", "trainable_params",
                "total_params", "training_samples", "validation_samples", "final_train_loss", "world_size",
                "distributed_training"}  # training.py:319-332
    assert ref_keys <= set(summary)
    assert summary["world_size"] == 1 and summary["training_samples"] == 2560 and summary["validation_samples"] == 285
    hist = json.load(open(out / "training_history.json"))
    assert any("loss" in h for h in hist) and any("eval_loss" in h for h in hist)
    # step-phase breakdown and GPU telemetry into the tracker (subset=system, O3)
    train_logs = [h for h in hist if "loss" in h]
    for k in ("data_ms", "fwd_ms", "bwd_ms", "comm_wait_ms", "optim_ms"):
        assert all(k in h and h[k] >= 0 for h in train_logs), k
    assert train_logs[0]["sys_gpu0_gfx_util"] == 97.0
    aim = [json.loads(l) for l in open(tmp_path / "aim" / "smollm3-wilderness-finetuning-distributed.jsonl")]
    assert {"name": "gpu0_power_w", "value": 812.0} == {k: next(r for r in aim if r["name"] == "gpu0_power_w")[k]
                                                        for k in ("name", "value")}
    assert next(r for r in aim if r["name"] == "gpu0_power_w")["context"] == {"subset": "system"}
    resolved = json.load(open(out / "sft_config.json"))
    assert resolved["eval_steps"] == 1 and resolved["warmup_steps"] == 1 and resolved["lr_scheduler_type"] == "cosine"
    assert resolved["max_length"] == 256
    best = out / "best_model"
    assert (best / "config.json").exists() and (best / "generation_config.json").exists()
    assert any(f.endswith(".safetensors") for f in os.listdir(best))
