"""Quick single-GPU fwd/bwd timing of SmolLM3-3B (random init) for early bring-up."""
import argparse
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import torch

from llm_fine_tune_distributed_amd.models import build_model, smollm3_3b

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--seq", type=int, default=512)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--layers", type=int, default=0)
a = ap.parse_args()
cfg = smollm3_3b()
if a.layers:
    cfg.num_hidden_layers = a.layers
t0 = time.time()
m = build_model(cfg, device="cuda", dtype=torch.bfloat16)
print(f"build {time.time()-t0:.1f}s params {m.num_parameters()/1e9:.3f}B", flush=True)
for p in m.parameters():
    p.main_grad = torch.zeros_like(p)
ids = torch.randint(0, cfg.vocab_size, (a.batch, a.seq), device="cuda")
for it in range(a.steps + 2):
    torch.cuda.synchronize()
    t = time.time()
    m.reset_grad_use_counters()
    out = m(ids, labels=ids)
    out.loss.backward()
    torch.cuda.synchronize()
    dt = time.time() - t
    tok = a.batch * a.seq
    fl = cfg.flops_per_token(a.seq) * tok
    print(f"it {it} loss {out.loss.item():.4f} {dt*1000:.1f} ms  {tok/dt:.0f} tok/s  {fl/dt/1e12:.0f} TFLOP/s", flush=True)
print("mem GB", torch.cuda.max_memory_allocated() / 1e9)
