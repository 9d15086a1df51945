#!/usr/bin/env python3
"""Headline benchmark: SmolLM3-3B full-parameter SFT, bf16, samples/s on N MI355X GPUs.

Metric and config follow BASELINE.json: "samples/sec SmolLM3-3B full SFT bf16 at 1/2/4/8
MI355X; DDP scaling efficiency", reference 4-GPU config = per-device batch 8 x GA 2
(README.md:69). Every timed step is a complete optimizer step of the real training path
(``SFTTrainer.optimizer_step``): GA micro-batches of fwd+bwd through the HIP kernels, RCCL
bucket reduce-scatter (ZeRO-1, default for N > 1) or all-reduce overlapped with backward, grad-norm
clip, fused AdamW (bf16 params + stochastic rounding, fp32 moments) and, with ZeRO-1, the parameter
all-gather (finished inside the timed region).
Data: synthetic token sequences of ``--seq`` tokens (the reference's samples are ~420-525
tokens), random-init weights of the SmolLM3-3B architecture (no network).

Weak scaling: per-GPU work is fixed (micro-batch x GA), global batch = 16 x N. With N > 1 the optimizer
state is sharded ZeRO-1 style by default (``--zero 0`` = replicated all-reduce DDP).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="smollm3-3b")
    # Reference 4-GPU config: 8 samples/device x GA 2 = 16 samples per device per optimizer step
    # (README.md:69). MI355X's 288 GB holds all 16 at once, so the default runs them as ONE
    # micro-batch (identical optimizer-step math: the loss is normalised by the step's global
    # token count either way); --micro-batch 8 --ga 2 reproduces the reference split.
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--ga", type=int, default=1)
    ap.add_argument("--no-overlap", action="store_true", help="disable AdamW/forward overlap")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("SFTAMD_BUCKET_MB", "64")))
    ap.add_argument("--packing", action="store_true")
    ap.add_argument("--freeze-policy", default="full", choices=["full", "last_n_layers", "lora"])
    ap.add_argument("--master-weights", action="store_true", help="fp32 master copy (default: bf16 params + SR)")
    ap.add_argument("--optim-state", default=os.environ.get("SFTAMD_OPTIM_STATE", "fp32"), choices=["fp32", "bf16"],
                    help="Adam moment dtype (bf16 = torch AdamW's state dtype for the reference's bf16 params)")
    ap.add_argument("--zero", type=int, default=int(os.environ.get("SFTAMD_ZERO", "1")), choices=[0, 1],
                    help="1 (default): ZeRO-1 over the DDP buckets when N > 1 (reduce-scatter grads, 1/N of AdamW "
                         "per rank, all-gather params under the next forward); 0: replicated all-reduce DDP")
    ap.add_argument("--tunableop", default=os.environ.get("SFTAMD_TUNABLEOP", "auto"),
                    help="auto: load the committed GEMM selections; tune: tune missing shapes into it; off")
    ap.add_argument("--profile-steps", type=int, default=0)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.models import build_model, get_config
    from llm_fine_tune_distributed_amd.parallel.process_group import barrier, setup_distributed
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer

    st = setup_distributed(verbose=False)
    if a.tunableop != "off" and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ:
        from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(tune=(a.tunableop == "tune"), verbose=st.is_main)
    if st.world_size != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={st.world_size}")
    cfg = get_config(a.model)
    model = build_model(cfg, device=st.device, dtype=torch.bfloat16, seed=0)
    per_rank_samples = a.micro_batch * a.ga * (a.steps + a.warmup + 2)
    ds = TokenizedDataset.synthetic(per_rank_samples * st.world_size, cfg.vocab_size, a.seq, a.seq, seed=1)
    args = SFTConfig(output_dir="/tmp/sftamd_bench", per_device_train_batch_size=a.micro_batch,
                     gradient_accumulation_steps=a.ga, learning_rate=5e-5 * st.world_size, max_grad_norm=1.0,
                     bf16=True, gradient_checkpointing=False, max_length=a.seq, packing=a.packing,
                     ddp_bucket_cap_mb=a.bucket_mb, dataloader_drop_last=True, jsonl_log=False, logging_steps=0,
                     optimizer_overlap=not a.no_overlap, freeze_policy=a.freeze_policy,
                     master_weights=a.master_weights, optim_state_dtype=a.optim_state,
                     shard_optimizer_state=bool(a.zero))
    trainer = SFTTrainer(model=model, args=args, train_dataset=ds)
    loader = trainer.get_train_dataloader()
    it = iter(loader)

    def next_micro():
        return [next(it) for _ in range(a.ga)]

    def step():
        return trainer.optimizer_step(next_micro(), lr=args.learning_rate)

    for _ in range(a.warmup):
        r = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=st.device, dtype=torch.float64)
    if st.world_size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    trainer.optimizer.synchronize()
    loss = r["acc"][0].item()
    ms = dt / a.steps * 1e3
    samples = a.micro_batch * a.ga * st.world_size * a.steps
    value = samples / dt
    tok_s = value * a.seq
    mfu = tok_s * cfg.flops_per_token(a.seq) / (2.5e15 * st.world_size) if a.freeze_policy == "full" else None
    if st.is_main:
        rec = {
            "metric": ("samples/sec SmolLM3-3B full SFT bf16 (DDP)" if a.model == "smollm3-3b" and a.freeze_policy == "full"
                       else f"samples/sec {a.model} {a.freeze_policy} SFT bf16 (DDP)"),
            "value": round(value, 3), "unit": "samples/s", "n_gpus": st.world_size, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": {"smollm3-3b": "SmolLM3-3B", "llama3-8b": "Llama-3-8B"}.get(a.model, a.model),
                       "freeze_policy": a.freeze_policy, "global_batch": a.micro_batch * a.ga * st.world_size,
                       "per_device_batch": a.micro_batch, "gradient_accumulation_steps": a.ga, "seq_len": a.seq,
                       "parallelism": f"dp{st.world_size}", "optimizer": ("AdamW fp32-master (fused HIP)" if a.master_weights else
                                     f"AdamW bf16 params + stochastic rounding, {a.optim_state} moments (fused HIP)"),
                       "samples_per_device_per_step": a.micro_batch * a.ga,
                       "optimizer_sharding": "zero1" if (a.zero and st.world_size > 1) else "none",
                       "gradient_checkpointing": False, "packing": a.packing},
            "tokens_per_sec": round(tok_s, 1), "mfu": None if mfu is None else round(mfu, 4), "final_loss": round(loss, 4),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2),
        }
        print(json.dumps(rec), flush=True)
    if a.profile_steps:
        torch.cuda.synchronize()
        for _ in range(a.profile_steps):
            step()
        torch.cuda.synchronize()
    if st.world_size > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
