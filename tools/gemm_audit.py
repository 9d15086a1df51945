"""Per-shape GEMM efficiency inside one full training step (SmolLM3-3B, 16 x 512, synthetic): torch.profiler
with input shapes over ``SFTTrainer.optimizer_step``; every matmul-like op (ATen mm/addmm/linear and the
sftamd HIP GEMMs) is listed with its shapes, calls, device time and achieved TFLOP/s.

    python tools/gemm_audit.py > gpurun_out/gemm_audit.txt
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
from torch.profiler import ProfilerActivity, profile

from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
from llm_fine_tune_distributed_amd.models import build_model, get_config
from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms

enable_tuned_gemms(tune=False, verbose=False)
cfg = get_config("smollm3-3b")
model = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=0)
ds = TokenizedDataset.synthetic(16 * 6, cfg.vocab_size, 512, 512, seed=1)
args = SFTConfig(output_dir="/tmp/sftamd_audit", per_device_train_batch_size=16, gradient_accumulation_steps=1,
                 learning_rate=5e-5, bf16=True, gradient_checkpointing=False, max_length=512,
                 dataloader_drop_last=True, jsonl_log=False, logging_steps=0, freeze_policy="full")
trainer = SFTTrainer(model=model, args=args, train_dataset=ds)
it = iter(trainer.get_train_dataloader())
for _ in range(3):
    trainer.optimizer_step([next(it)], lr=args.learning_rate)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    trainer.optimizer_step([next(it)], lr=args.learning_rate)
    torch.cuda.synchronize()


def flops(name, shapes):
    try:
        if name in ("aten::mm",):
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2 * m * n * k
        if name == "aten::addmm":
            (m, k), (_, n) = shapes[1], shapes[2]
            return 2 * m * n * k
        if name == "aten::linear":
            x, w = shapes[0], shapes[1]
            m = 1
            for d in x[:-1]:
                m *= d
            return 2 * m * w[0] * w[1]
        if name.startswith("sftamd::gemm_tn"):
            (m, k), (n, _) = shapes[0], shapes[1]
            return 2 * m * n * k
        if name == "sftamd::dgrad_gemm":  # dy [M, K], w [K, N]
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2 * m * n * k
        if name == "sftamd::wgrad_gemm":  # out [N, K], dy [T, N], x [T, K]
            (n, k), (t, _) = shapes[0], shapes[1]
            return 2 * t * n * k
    except Exception:
        return None
    return None


rows = []
for e in prof.key_averages(group_by_input_shape=True):
    if not (e.key in ("aten::mm", "aten::addmm") or e.key.startswith("sftamd::gemm_tn")
            or e.key in ("sftamd::wgrad_gemm", "sftamd::dgrad_gemm")):
        continue
    dev = getattr(e, "device_time_total", None)
    if dev is None:
        dev = getattr(e, "cuda_time_total", 0)
    if dev <= 0:
        continue
    f = flops(e.key, e.input_shapes)
    tf = f * e.count / (dev * 1e-6) / 1e12 if f else float("nan")
    rows.append((dev, e.count, e.key, e.input_shapes, tf))
rows.sort(key=lambda r: -r[0])
tot = sum(r[0] for r in rows)
print(f"GEMM device time in one step: {tot / 1e3:.2f} ms")
print(f"{'ms':>8} {'calls':>5} {'TF/s':>6}  op  shapes")
for dev, n, key, shp, tf in rows:
    print(f"{dev / 1e3:8.2f} {n:5d} {tf:6.0f}  {key}  {shp}")
