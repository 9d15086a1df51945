"""Find the non-sftamd device work inside one full training step (copies, fills, ATen elementwise):
torch.profiler over ``SFTTrainer.optimizer_step`` on SmolLM3-3B (random init, synthetic 16 x 512), grouped by
op + Python stack so each copy / fill is traced back to its call site.

    python tools/copy_audit.py [--micro-batch 16] [--seq 512] > gpurun_out/copy_audit.txt
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
from torch.profiler import ProfilerActivity, profile

from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
from llm_fine_tune_distributed_amd.models import build_model, get_config
from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms

ap = argparse.ArgumentParser()
ap.add_argument("--micro-batch", type=int, default=16)
ap.add_argument("--seq", type=int, default=512)
ap.add_argument("--model", default="smollm3-3b")
a = ap.parse_args()

enable_tuned_gemms(tune=False, verbose=False)
cfg = get_config(a.model)
model = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=0)
ds = TokenizedDataset.synthetic(a.micro_batch * 6, cfg.vocab_size, a.seq, a.seq, seed=1)
args = SFTConfig(output_dir="/tmp/sftamd_audit", per_device_train_batch_size=a.micro_batch,
                 gradient_accumulation_steps=1, learning_rate=5e-5, bf16=True, gradient_checkpointing=False,
                 max_length=a.seq, dataloader_drop_last=True, jsonl_log=False, logging_steps=0, freeze_policy="full")
trainer = SFTTrainer(model=model, args=args, train_dataset=ds)
it = iter(trainer.get_train_dataloader())
for _ in range(3):
    trainer.optimizer_step([next(it)], lr=args.learning_rate)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    trainer.optimizer_step([next(it)], lr=args.learning_rate)
    torch.cuda.synchronize()

keys = ("copy_", "fill_", "zero_", "clone", "contiguous", "to", "cat", "add", "mul", "sort", "index", "cos", "sin",
        "arange", "searchsorted", "sum", "where", "masked", "stack", "div", "sqrt", "clamp", "empty_like", "zeros")
rows = []
for e in prof.key_averages(group_by_stack_n=6):
    name = e.key
    if name.startswith("sftamd::") or not any(k in name for k in keys):
        continue
    dev_us = getattr(e, "self_device_time_total", None)
    if dev_us is None:
        dev_us = getattr(e, "self_cuda_time_total", 0)
    if dev_us <= 0:
        continue
    rows.append((dev_us, e.count, name, e.stack))
rows.sort(key=lambda r: -r[0])
total = sum(r[0] for r in rows)
print(f"non-sftamd device time in one step (ATen ops matched): {total / 1e3:.2f} ms")
for dev_us, n, name, stack in rows[:40]:
    print(f"\n{dev_us / 1e3:8.3f} ms  x{n:4d}  {name}")
    for fr in (stack or [])[:6]:
        if "site-packages" not in fr:
            print(f"            {fr}")
