"""Reference-compatible training entrypoint (``training.py`` equivalent).

Same env contract (EPOCHS, BATCH_SIZE, LEARNING_RATE, DATA_DIR, OUTPUT_DIR, AIM_REPO; WORLD_SIZE/RANK/...),
same SFTConfig values (GA 4, eval every 10 steps, logging every 2, clip 1.0, LR x world size,
best-by-eval_loss, save every 500 / keep 3), same callbacks (history, perplexity, Aim) and the same
rank-0 artifacts: ``best_model/`` (HF safetensors + tokenizer), ``training_history.json``,
``training_summary.json``. Runs on CPU/gloo too (the reference hard-fails without CUDA).

    python -m llm_fine_tune_distributed_amd.launch --nproc-per-node 8 -m llm_fine_tune_distributed_amd.cli.train
"""
from __future__ import annotations

import argparse
import json
import os

import torch


def main(argv=None):
    from ..data.dataset import load_jsonl, load_qa_parquet, train_test_split
    from ..data.prompts import format_prompt
    from ..data.synthetic import generate_qa
    from ..data.tokenizer import load_tokenizer
    from ..parallel.process_group import cleanup_distributed, setup_distributed
    from ..train import (AimCallback, PerplexityCallback, SFTConfig, SFTTrainer, TrainingHistoryCallback,
                         config_from_env)
    from ..train.config import apply_overrides

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=os.getenv("MODEL_NAME", "HuggingFaceTB/SmolLM3-3B"),
                    help="preset name or local HF directory (config.json + safetensors)")
    ap.add_argument("--dataset", default=os.getenv("DATASET_PATH", "data/qa_dataset.parquet"),
                    help="parquet/jsonl Q&A file; 'synthetic' (or a missing file) generates the synthetic set")
    ap.add_argument("--freeze-policy", default=os.getenv("FREEZE_POLICY", "last_n_layers"),
                    choices=["last_n_layers", "full", "lora"])
    ap.add_argument("--grad-accum", type=int, default=int(os.getenv("GRAD_ACCUM", "4")))
    ap.add_argument("--max-steps", type=int, default=-1)
    ap.add_argument("--max-length", type=int, default=1024)
    ap.add_argument("--packing", action="store_true")
    ap.add_argument("--lr-scheduler", default="linear")
    ap.add_argument("--no-gradient-checkpointing", action="store_true")
    ap.add_argument("--resume", default=None, help="checkpoint dir or 'auto'")
    ap.add_argument("--max-train-samples", type=int, default=None)
    ap.add_argument("--log-step-phases", action="store_true",
                    help="log data/fwd/bwd/comm_wait/optim *_ms per step (roctx ranges around each phase)")
    ap.add_argument("--log-system-metrics-every", type=int, default=int(os.getenv("LOG_SYSTEM_METRICS_EVERY", "0")),
                    help="GPU telemetry (amdsmi) into the trackers every N log steps (0 = off)")
    ap.add_argument("--config", default=os.getenv("SFT_CONFIG"),
                    help="YAML/JSON file of SFTConfig field overrides (applied over the reference defaults)")
    ap.add_argument("--set", dest="sets", action="append", default=[], metavar="FIELD=VALUE",
                    help="override one SFTConfig field (repeatable; highest precedence)")
    ap.add_argument("--merge-lora", action="store_true",
                    help="LoRA runs: write best_model/ with the adapters merged into the weights")
    a = ap.parse_args(argv)

    st = setup_distributed()
    env = config_from_env(world_size=st.world_size)
    out = env["output_dir"]
    if st.is_main:
        os.makedirs(f"{out}/best_model", exist_ok=True)
        print("Configuration:")
        for k in ("epochs", "batch_size", "learning_rate", "data_dir", "output_dir"):
            print(f"- {k}: {env[k]}")
        print(f"- model: {a.model}\n- dataset: {a.dataset}\n- device: {st.device}")

    # dataset (training.py:155-212)
    if a.dataset != "synthetic" and os.path.exists(a.dataset):
        rows = load_qa_parquet(a.dataset) if a.dataset.endswith(".parquet") else load_jsonl(a.dataset)
    else:
        rows = generate_qa(2845, seed=42)
        rows = [{"full-question": r["full-question"], "answer": r["answer"]} for r in rows]
    train_rows, val_rows = train_test_split(rows, test_size=0.1, seed=42)
    if st.is_main:
        print(f"Total dataset size: {len(rows):,} | train {len(train_rows):,} | val {len(val_rows):,}")
    train_rows = [format_prompt(r) for r in train_rows]
    val_rows = [format_prompt(r) for r in val_rows]
    tok_dir = a.model if os.path.isdir(a.model) else None
    tokenizer = load_tokenizer(tok_dir)

    history, ppl = TrainingHistoryCallback(), PerplexityCallback()
    aim = AimCallback(repo=env["aim_repo"], experiment="smollm3-wilderness-finetuning-distributed")
    dist_args = {}
    if st.world_size > 1:
        # the reference's ddp_bucket_cap_mb=50 (training.py:253) was sized for one TCP ring; on the xGMI
        # full mesh the cap grows with N (parallel/ddp.py plan_bucket_mb). DDP_BUCKET_CAP_MB pins it.
        cap = float(os.environ["DDP_BUCKET_CAP_MB"]) if os.environ.get("DDP_BUCKET_CAP_MB") else None
        dist_args = dict(ddp_find_unused_parameters=False, ddp_bucket_cap_mb=cap, local_rank=st.local_rank)
    args = SFTConfig(
        output_dir=f"{out}/checkpoints", per_device_train_batch_size=env["batch_size"],
        per_device_eval_batch_size=env["batch_size"], gradient_accumulation_steps=a.grad_accum,
        learning_rate=env["scaled_learning_rate"], max_grad_norm=1.0, num_train_epochs=env["epochs"],
        max_steps=a.max_steps, logging_steps=2, logging_first_step=True, save_steps=500, bf16=True,
        eval_strategy="steps", eval_steps=10, save_strategy="steps", load_best_model_at_end=True,
        metric_for_best_model="eval_loss", greater_is_better=False, save_total_limit=3, dataloader_pin_memory=True,
        dataloader_num_workers=0, remove_unused_columns=False,
        gradient_checkpointing=not a.no_gradient_checkpointing, dataloader_drop_last=True,
        max_seq_length=a.max_length, packing=a.packing, ddp_backend="nccl" if st.device.type == "cuda" else "gloo",
        freeze_policy=a.freeze_policy, lr_scheduler_type=a.lr_scheduler, max_train_samples=a.max_train_samples,
        log_step_phases=a.log_step_phases, log_system_metrics_every=a.log_system_metrics_every,
        **dist_args)
    args = apply_overrides(args, a.config, a.sets)
    if st.is_main:  # the resolved configuration of this run, next to its artifacts
        args.to_json(f"{out}/sft_config.json")
    trainer = SFTTrainer(model=a.model, args=args, train_dataset=train_rows, eval_dataset=val_rows,
                         processing_class=tokenizer, callbacks=[history, ppl, aim])
    if st.device.type == "cuda" and st.is_main:
        print(f"VRAM after model load: {torch.cuda.memory_allocated() / 2**30:.2f} GB allocated")
    result = trainer.train(resume_from_checkpoint=a.resume)

    trainer.save_model(f"{out}/best_model", merge_lora=a.merge_lora)  # rank 0 writes, all ranks barrier
    if st.is_main:
        with open(f"{out}/training_history.json", "w") as f:
            json.dump(history.history, f, indent=2)
        summary = {
            "model_name": a.model, "dataset_path": a.dataset, "epochs": env["epochs"], "batch_size": env["batch_size"],
            "learning_rate": env["learning_rate"], "trainable_params": trainer.trainable_params,
            "total_params": trainer.total_params, "training_samples": len(train_rows),
            "validation_samples": len(val_rows), "final_train_loss": result.training_loss,
            "world_size": st.world_size, "distributed_training": st.world_size > 1,
            # MI355X-native additions
            "train_samples_per_second": result.metrics["train_samples_per_second"],
            "train_pure_samples_per_second": result.metrics["train_pure_samples_per_second"],
            "train_tokens_per_second": result.metrics["train_tokens_per_second"],
            "train_mfu": result.metrics["train_mfu"],
        }
        with open(f"{out}/training_summary.json", "w") as f:
            json.dump(summary, f, indent=2)
        print(f"\nDistributed Q&A fine-tuning completed successfully!\nArtifacts saved to {out}/\n"
              f"World size: {st.world_size}")
    cleanup_distributed()


if __name__ == "__main__":
    main()
