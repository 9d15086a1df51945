"""Hunt an intermittent non-finite loss: the bench's training step (same model, data, SFTConfig) run for a few steps,
with a full finiteness check after every step — loss, every parameter's gradient, the parameters and the Adam
moments — and, on the first failure, which parameters went bad. Repeats the whole run (fresh model) R times.

    python tools/nan_hunt.py [--model llama3-8b] [--steps 13] [--reps 4] [--no-overlap]
"""
import argparse
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset  # noqa: E402
from llm_fine_tune_distributed_amd.models import build_model, get_config  # noqa: E402
from llm_fine_tune_distributed_amd.parallel.process_group import setup_distributed  # noqa: E402
from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer  # noqa: E402
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402


def bad_params(trainer, which):
    out = []
    for name, p in trainer.model.named_parameters():
        t = p.main_grad if which == "grad" else p.data
        if t is not None and not torch.isfinite(t).all():
            out.append(f"{name}({int((~torch.isfinite(t)).sum())})")
    return out


def run(a, rep):
    cfg = get_config(a.model)
    model = build_model(cfg, device=a.dev, dtype=torch.bfloat16, seed=0)
    n = a.batch * (a.steps + 2)
    ds = TokenizedDataset.synthetic(n, cfg.vocab_size, a.seq, a.seq, seed=1)
    args = SFTConfig(output_dir="/tmp/sftamd_nan", per_device_train_batch_size=a.batch, gradient_accumulation_steps=1,
                     learning_rate=5e-5, max_grad_norm=1.0, bf16=True, gradient_checkpointing=False,
                     max_length=a.seq, dataloader_drop_last=True, jsonl_log=False, logging_steps=0,
                     optimizer_overlap=not a.no_overlap, freeze_policy="full", gemm_tuning=False)
    trainer = SFTTrainer(model=model, args=args, train_dataset=ds)
    it = iter(trainer.get_train_dataloader())
    eng, opt = trainer.engine, trainer.optimizer
    for s in range(1, a.steps + 1):
        r = trainer.optimizer_step([next(it)], lr=args.learning_rate)
        # only the loss / grad norm each step (a main-stream sync): the overlapped update keeps running under the
        # next forward, as in the bench; the full check after a failure or at the end
        loss = float(r["acc"][0])
        gn = r.get("grad_norm")
        gn = float(gn) if gn is not None else float("nan")
        ok = loss == loss and gn == gn and abs(loss) != float("inf")
        last = not ok or s == a.steps
        fin = {}
        if last:
            opt.synchronize()
            if a.dev.type == "cuda":
                torch.cuda.synchronize()
            fin = {"grads": bool(torch.isfinite(eng.grad_flat).all()),
                   "params": bool(torch.isfinite(eng.param_flat).all()),
                   "m": bool(torch.isfinite(opt.exp_avg).all()) if hasattr(opt, "exp_avg") else True,
                   "v": bool(torch.isfinite(opt.exp_avg_sq).all()) if hasattr(opt, "exp_avg_sq") else True}
            ok = ok and all(fin.values())
        print(f"rep {rep} step {s}: loss {loss:.4f} grad_norm {gn:.4g} {fin}", flush=True)
        if not ok:
            print(f"rep {rep} FIRST NON-FINITE at step {s}: grads {bad_params(trainer, 'grad')[:12]} "
                  f"params {bad_params(trainer, 'param')[:12]}", flush=True)
            break
    del trainer, model, it, eng, opt
    gc.collect()
    if a.dev.type == "cuda":
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--steps", type=int, default=13)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    a.dev = setup_distributed(verbose=False, device=a.device).device
    if a.dev.type == "cuda":
        enable_tuned_gemms()
    for rep in range(a.reps):
        run(a, rep)


if __name__ == "__main__":
    main()
