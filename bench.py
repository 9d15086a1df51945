#!/usr/bin/env python3
"""Headline benchmark: SmolLM3-3B full-parameter SFT, bf16, samples/s on N MI355X GPUs.

Metric and config follow BASELINE.json: "samples/sec SmolLM3-3B full SFT bf16 at 1/2/4/8
MI355X; DDP scaling efficiency", reference 4-GPU config = per-device batch 8 x GA 2
(README.md:69). Every timed step is a complete optimizer step of the real training path
(``SFTTrainer.optimizer_step``): GA micro-batches of fwd+bwd through the HIP kernels, RCCL
bucket reduce-scatter (ZeRO-1, default for N > 1) or all-reduce overlapped with backward, grad-norm
clip, fused AdamW (bf16 params and bf16 moments like the reference's torch AdamW over its bf16 model, both
stochastically rounded) and, with ZeRO-1, the parameter
all-gather (finished inside the timed region).
Data: synthetic token sequences of ``--seq`` tokens (the reference's samples are ~420-525
tokens), random-init weights of the SmolLM3-3B architecture (no network).

Weak scaling: per-GPU work is fixed (micro-batch x GA), global batch = 16 x N. With N > 1 the optimizer
state is sharded ZeRO-1 style by default (``--zero 0`` = replicated all-reduce DDP).

Launching (the reference's ``training.py:16-42`` env contract):

    python bench.py [--gpus N] [--steps K] [--warmup W]          # N > 1: spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    python bench.py --gpus 4 --device cpu --model tiny             # gloo rehearsal of the N-rank path

When ``WORLD_SIZE`` is unset and ``--gpus N > 1`` this process becomes a launcher: it never imports
torch (so it never touches a GPU), starts N fresh ``bench.py`` children with the torchrun env contract
(``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT``) through ``launch.py``, lets rank 0
print the JSON line, and exits with the first failing rank's code after tearing the others down.

Besides the driver contract fields the JSON line carries the multi-GPU diagnostics a scaling run needs:
``dist`` (backend and world size as every rank saw them), ``bucket_plan`` (count / sizes of the
gradient buckets), ``comm_exposed_ms`` (non-overlapped gradient-collective wait per step, max over
ranks), per-rank ``peak_mem_gb`` / ``ms_per_step`` and, given ``--baseline-1gpu V``,
``scaling_efficiency = value / (N * V)``. ``comm_probe`` (N > 1, measured between warmup and the timed steps):
reduce-scatter / all-gather / all-reduce bus bandwidth at the bucket size, i.e. what xGMI delivered on that node.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="smollm3-3b")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="cpu: gloo + the PyTorch fallbacks (a CPU rehearsal of the N-rank path; use --model tiny)")
    # Reference 4-GPU config: 8 samples/device x GA 2 = 16 samples per device per optimizer step
    # (README.md:69). MI355X's 288 GB holds all 16 at once, so the default runs them as ONE
    # micro-batch (identical optimizer-step math: the loss is normalised by the step's global
    # token count either way); --micro-batch 8 --ga 2 reproduces the reference split.
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--ga", type=int, default=1)
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="AdamW / ZeRO-1 gathers under the next forward on a side stream: auto = on for N > 1 (hides "
                         "the parameter all-gathers), off for one GPU (the overlapped update slowed the step by 1 %%: "
                         "112.7 / 112.5 vs 113.8 / 113.6 samples/s, profiles/r6_adamw_overlap.md)")
    ap.add_argument("--no-overlap", action="store_true", help="= --overlap off")
    ap.add_argument("--ga-merge-max-tokens", type=int, default=None,
                    help="run the GA micro-batches of a step as one pass up to this many tokens (SFTConfig default "
                         "32768); 0 = one fwd/bwd pass per micro-batch")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--bucket-mb", type=float, default=0.0,
                    help="gradient bucket cap in MB; 0 (default) = the xGMI plan of parallel.ddp.plan_bucket_mb")
    ap.add_argument("--packing", action="store_true")
    ap.add_argument("--padding-free", choices=["auto", "on", "off"], default="auto",
                    help="SFTConfig.padding_free (auto: the trainer default, on for GPU training)")
    ap.add_argument("--freeze-policy", default="full", choices=["full", "last_n_layers", "lora"])
    ap.add_argument("--master-weights", action="store_true", help="fp32 master copy (default: bf16 params + SR)")
    ap.add_argument("--optim-state", default="bf16", choices=["fp32", "bf16"],
                    help="Adam moment dtype. bf16 (default) = the reference's: torch AdamW keeps exp_avg / exp_avg_sq "
                         "in the parameter dtype, bf16 for its bf16 model (training.py:99); here stored with "
                         "stochastic rounding (unbiased), so not less precise than the reference")
    ap.add_argument("--zero", type=int, default=1, choices=[0, 1],
                    help="1 (default): ZeRO-1 over the DDP buckets when N > 1 (reduce-scatter grads, 1/N of AdamW "
                         "per rank, all-gather params under the next forward); 0: replicated all-reduce DDP")
    ap.add_argument("--tunableop", default="auto",
                    help="auto: load the committed GEMM selections; tune: tune missing shapes into it; off")
    ap.add_argument("--baseline-1gpu", type=float, default=0.0,
                    help="1-GPU samples/s of the same config: adds scaling_efficiency = value / (N * this)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--torch-profile", default="",
                    help="with --profile-steps: record those steps with torch.profiler and write the ops by device "
                         "time (with input shapes) to this file (attributes small copy / fill kernels to their op)")
    # --recipe: the reference recipe end to end instead of the synthetic step loop: its own parquet
    # (data/qa_dataset.parquet, 90/10 split, system prompt + chat template), per-device batch 8 x GA 2 (README.md:69),
    # eval every 10 steps, through SFTTrainer.train(); reports HF's train_samples_per_second (wall time INCLUDING the
    # evals, BASELINE.md "Metric definition") as value, and the pure-training samples/s next to it
    ap.add_argument("--recipe", action="store_true", help="reference parquet + evals through SFTTrainer.train()")
    ap.add_argument("--dataset", default=os.path.join(HERE, "data", "qa_dataset.parquet"))
    ap.add_argument("--eval-steps", type=int, default=10)
    ap.add_argument("--eval-batch", type=int, default=32,
                    help="--recipe: per-device eval batch (eval loss is token-weighted, independent of it)")
    # hang protection for the first RCCL multi-rank runs (utils/heartbeat.py, launch.py): a wall-clock bound on the
    # whole run, a no-progress bound per rank (also the process group's collective timeout), and RCCL INFO capture
    # (default at N > 1 on GPUs, --no-rccl-info to opt out) whose channel / transport / rank-count summary lands in the
    # JSON line's ``dist``
    ap.add_argument("--timeout-s", type=float, default=900.0,
                    help="wall-clock limit of the whole run; on expiry every rank prints its last heartbeat and exits 124")
    ap.add_argument("--hang-timeout-s", type=float, default=300.0,
                    help="seconds without progress (no heartbeat) before a rank is declared hung")
    ap.add_argument("--no-rccl-info", action="store_true", help="N > 1: do not capture RCCL's INFO log")
    ap.add_argument("--rccl-log-dir", default="/tmp/sftamd_rccl")
    ap.add_argument("--no-comm-probe", action="store_true", help="N > 1: skip the post-warmup collective probe")
    ap.add_argument("--no-strict-dist", action="store_true",
                    help="N > 1 on GPUs: still exit 0 when RCCL's log shows a degraded path (non-P2P transport, rank "
                         "count mismatch, failed init, fewer channels than peer links); by default the JSON line is "
                         "printed with dist.warnings and the run exits 3")
    return ap.parse_args(argv)


def launch_ranks(a, argv) -> int:
    """Parent side of a standalone ``--gpus N`` run: spawn N ranks, never touch the GPU.

    ``launch.py`` is loaded by file path so the package ``__init__`` (which imports torch) does not run
    here; its children stay in this process group and die with this process (PR_SET_PDEATHSIG)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_sftamd_launch", os.path.join(HERE, "llm_fine_tune_distributed_amd", "launch.py"))
    launch = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(launch)
    return launch.run(["--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1", "--same-session",
                       "--grace", "15", "--hang-timeout", str(a.hang_timeout_s), "--deadline", str(a.timeout_s + 60),
                       os.path.abspath(__file__)] + list(argv))


def bucket_plan(engine) -> dict:
    mb = [(b.end - b.start) * engine.grad_flat.element_size() / 2 ** 20 for b in engine.buckets]
    srt = sorted(mb)
    return {"count": len(mb), "cap_mb": round(engine.bucket_cap_mb, 3), "first_mb": round(mb[0], 3),
            "min_mb": round(srt[0], 3), "median_mb": round(srt[len(srt) // 2], 3), "max_mb": round(srt[-1], 3),
            "total_mb": round(sum(mb), 1), "split_params": engine.num_split_params,
            "tied_sparse": bool(getattr(engine, "tied_sparse", False)),
            "replicated_buckets": sum(bool(getattr(b, "replicated", False)) for b in engine.buckets),
            "plan_source": getattr(engine, "plan_source", None), "alpha_us": round(getattr(engine, "link_alpha_us", 0), 2),
            "link_gbps": round(getattr(engine, "link_gbps", 0), 2)}


def comm_probe(dev, world: int, nbytes: int, iters: int = 5) -> dict:
    """Bus bandwidth of the three collectives the step uses, at the gradient-bucket size, measured between the
    warmup and the timed steps (not timed): reduce-scatter and all-gather (ZeRO-1) and all-reduce (DDP), bf16.
    busbw = bytes / time x (N - 1) / N, the per-rank link traffic rate (nccl-tests convention)."""
    import torch
    import torch.distributed as dist
    n = max(world * 64, (nbytes // 2) // (world * 64) * (world * 64))
    buf = torch.ones(n, dtype=torch.bfloat16, device=dev)
    rank = dist.get_rank()
    part = buf[rank * (n // world):(rank + 1) * (n // world)]  # in place, as the ZeRO-1 buckets do
    out = {"bytes": n * 2}
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    for name, fn in (("reduce_scatter", lambda: dist.reduce_scatter_tensor(part, buf)),
                     ("all_gather", lambda: dist.all_gather_into_tensor(buf, part)),
                     ("all_reduce", lambda: dist.all_reduce(buf))):
        for _ in range(2):
            fn()
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        dt = (time.perf_counter() - t0) / iters
        bus = n * 2 / dt * (world - 1) / world * (2 if name == "all_reduce" else 1)
        out[f"{name}_ms"] = round(dt * 1e3, 3)
        out[f"{name}_busbw_gbps"] = round(bus / 1e9, 1)
    return out


def run(a):
    # watchdog of this rank (also under an external torchrun): no heartbeat for hang_timeout_s, or the whole run past
    # timeout_s -> print the last heartbeat, exit 124 (instead of waiting out the 1800 s process-group default)
    os.environ.setdefault("SFTAMD_HANG_TIMEOUT_S", str(a.hang_timeout_s))
    os.environ.setdefault("SFTAMD_RUN_DEADLINE_S", str(a.timeout_s))
    rccl_dir = None
    # N > 1: RCCL's INFO log is captured by default (--no-rccl-info opts out), so the first multi-GPU record says which
    # transport / how many channels each rank's communicator got and how many ranks RCCL saw
    if not a.no_rccl_info and int(os.environ.get("WORLD_SIZE", "1")) > 1 and a.device != "cpu":
        from llm_fine_tune_distributed_amd.parallel import rccl_info
        rccl_dir = a.rccl_log_dir
        rccl_info.enable(rccl_dir)
    import torch
    import torch.distributed as dist

    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    from llm_fine_tune_distributed_amd.models import build_model, get_config
    from llm_fine_tune_distributed_amd.parallel.process_group import barrier, setup_distributed
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer

    # the collective timeout sits above the watchdog's, so a stuck collective is reported by the heartbeat watchdog
    # (last position of this rank, exit 124) rather than by the process group's own abort
    st = setup_distributed(verbose=False, device="cpu" if a.device == "cpu" else None,
                           timeout_s=a.hang_timeout_s + 60)
    from llm_fine_tune_distributed_amd.utils import heartbeat as hb
    beat = hb.install(hb.Heartbeat(st.rank)).beat
    beat(0, "init")
    on_gpu = st.device.type == "cuda"
    if a.device == "cuda" and not on_gpu:
        raise SystemExit("--device cuda but no GPU is visible")
    if on_gpu and a.tunableop != "off" and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ:
        from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(tune=(a.tunableop == "tune"), verbose=st.is_main)
    if st.world_size != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={st.world_size}")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    cfg = get_config(a.model)
    model = build_model(cfg, device=st.device, dtype=torch.bfloat16, seed=0)
    per_rank_samples = a.micro_batch * a.ga * (a.steps + a.warmup + a.profile_steps + 2)
    ds = TokenizedDataset.synthetic(per_rank_samples * st.world_size, cfg.vocab_size, a.seq, a.seq, seed=1)
    args = SFTConfig(output_dir="/tmp/sftamd_bench", per_device_train_batch_size=a.micro_batch,
                     gradient_accumulation_steps=a.ga, learning_rate=5e-5 * st.world_size, max_grad_norm=1.0,
                     bf16=True, gradient_checkpointing=False, max_length=a.seq, packing=a.packing,
                     padding_free={"auto": None, "on": True, "off": False}[a.padding_free],
                     ddp_bucket_cap_mb=a.bucket_mb or None, dataloader_drop_last=True, jsonl_log=False,
                     logging_steps=0, optimizer_overlap=_overlap_arg(a), freeze_policy=a.freeze_policy,
                     master_weights=a.master_weights, optim_state_dtype=a.optim_state,
                     shard_optimizer_state=bool(a.zero), gemm_tuning=False,
                     **({} if a.ga_merge_max_tokens is None else {"ga_merge_max_tokens": a.ga_merge_max_tokens}))
    trainer = SFTTrainer(model=model, args=args, train_dataset=ds)
    loader = trainer.get_train_dataloader()
    it = iter(loader)

    from llm_fine_tune_distributed_amd.utils.faults import maybe_inject, nan_injection
    n_step = [0]
    # diagnostic (not a benchmark setting): SFTAMD_BENCH_HOG_CUS=R holds R CUs on a side stream for the first
    # SFTAMD_BENCH_HOG_US (default 100 ms) of every step — a one-GPU stand-in for the RCCL channel blocks that sit on
    # CUs while collectives overlap compute at N > 1 (tools/bench_cu_contention.py, profiles/r6_cu_contention.md)
    hog_cus = int(os.environ.get("SFTAMD_BENCH_HOG_CUS", "0")) if on_gpu else 0
    if hog_cus > 0:
        from llm_fine_tune_distributed_amd.ops import _ext as _hx
        hog_stream = torch.cuda.Stream()
        hog_sink = torch.zeros(256, device=st.device, dtype=torch.int32)
        hog_us = float(os.environ.get("SFTAMD_BENCH_HOG_US", "100000"))

    def step():
        n_step[0] += 1
        if hog_cus > 0:
            with torch.cuda.stream(hog_stream):
                _hx.ops().cu_hog(hog_sink, hog_cus, hog_us)
        maybe_inject(st.rank, n_step[0])  # SFTAMD_FAULT_INJECT=rank:step (launcher teardown test)
        if nan_injection(st.rank, n_step[0]):  # SFTAMD_FAULT_INJECT=rank:step:nan (the non-finite-loss exit test)
            with torch.no_grad():
                trainer.engine.param_flat.view(-1)[0] = float("nan")
        return trainer.optimizer_step([next(it) for _ in range(a.ga)], lr=args.learning_rate)

    beat(0, "warmup")
    for _ in range(a.warmup):
        r = step()
    trainer.optimizer.synchronize()
    sync()
    beat(None, "warmup_done")
    probe = None
    if st.world_size > 1 and not a.no_comm_probe:
        probe = comm_probe(st.device, st.world_size, int(trainer.engine.bucket_cap_mb * 2 ** 20))
    barrier()
    sync()
    trainer.engine.comm_exposed_ms(reset=True)  # drop the warmup's samples
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = step()
    trainer.optimizer.synchronize()  # ZeRO-1: the last step's parameter all-gathers land inside the timing
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    comm_ms = trainer.engine.comm_exposed_ms(reset=True)
    beat(None, "timed_done")
    peak = torch.cuda.max_memory_allocated() / 1e9 if on_gpu else 0.0
    mine = {"rank": st.rank, "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "device": str(st.device), "ms_per_step": round(dt / a.steps * 1e3, 3), "peak_mem_gb": round(peak, 2),
            "comm_exposed_ms": round(comm_ms, 3),
            # after the timed steps (untimed): every rank must hold bitwise the same parameters (DDP / ZeRO-1 gather)
            "param_sum": float(torch.sum(trainer.engine.param_flat, dtype=torch.float64))}
    if rccl_dir is not None:
        from llm_fine_tune_distributed_amd.parallel import rccl_info
        mine["rccl"] = rccl_info.summarize(rccl_dir)
    ranks = [mine]
    if st.world_size > 1:
        ranks = [None] * st.world_size
        dist.all_gather_object(ranks, mine)
    dt = max(r_["ms_per_step"] for r_ in ranks) * a.steps / 1e3  # the MAX over ranks
    loss_t = r["acc"][0].detach().clone().reshape(1)  # this rank's share of the global token-mean loss
    if st.world_size > 1:
        dist.all_reduce(loss_t)
    loss = loss_t.item()
    ms = dt / a.steps * 1e3
    samples = a.micro_batch * a.ga * st.world_size * a.steps
    value = samples / dt
    tok_s = value * a.seq
    full = a.freeze_policy == "full"
    mfu = tok_s * cfg.flops_per_token(a.seq) / (2.5e15 * st.world_size) if (full and on_gpu) else None
    shard = trainer.engine.shard
    dist_warn, fatal = [], False
    if st.world_size > 1 and rccl_dir is not None:
        from llm_fine_tune_distributed_amd.parallel import rccl_info
        dist_warn, fatal = rccl_info.dist_warnings([r_.get("rccl") for r_ in ranks], st.world_size)
    if st.world_size > 1 and len({_sum_key(r_["param_sum"]) for r_ in ranks}) != 1:
        dist_warn.append("parameters differ across ranks after the timed steps")
        fatal = True
    strict = st.world_size > 1 and not a.no_strict_dist
    if st.is_main:
        rec = {
            "metric": ("samples/sec SmolLM3-3B full SFT bf16 (DDP)" if a.model == "smollm3-3b" and full
                       else f"samples/sec {a.model} {a.freeze_policy} SFT bf16 (DDP)"),
            "value": round(value, 3), "unit": "samples/s", "n_gpus": st.world_size, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)" + ("" if on_gpu else "; CPU/gloo rehearsal"),
            "config": {"model": {"smollm3-3b": "SmolLM3-3B", "llama3-8b": "Llama-3-8B"}.get(a.model, a.model),
                       "freeze_policy": a.freeze_policy, "global_batch": a.micro_batch * a.ga * st.world_size,
                       "per_device_batch": a.micro_batch, "gradient_accumulation_steps": a.ga, "seq_len": a.seq,
                       "parallelism": f"dp{st.world_size}",
                       "optimizer": ("AdamW fp32-master" if a.master_weights else
                                     f"AdamW bf16 params + stochastic rounding, {a.optim_state} moments")
                       + (" (fused HIP)" if on_gpu else " (torch fallback)"),
                       "samples_per_device_per_step": a.micro_batch * a.ga,
                       "ga_passes_per_step": 1 if (a.ga > 1 and a.micro_batch * a.ga * a.seq <= args.ga_merge_max_tokens)
                       else a.ga,
                       "optimizer_sharding": "zero1" if shard else "none",
                       "gradient_checkpointing": False, "packing": a.packing,
                       "padding_free": bool(getattr(trainer, "packed", False)) and not a.packing},
            "tokens_per_sec": round(tok_s, 1), "mfu": None if mfu is None else round(mfu, 4),
            "final_loss": round(loss, 4), "loss_finite": math.isfinite(loss),
            "peak_mem_gb": max(r_["peak_mem_gb"] for r_ in ranks),
            "dist": {"backend": mine["backend"], "world_size": mine["world_size"],
                     "consistent": all(r_["world_size"] == st.world_size and r_["backend"] == mine["backend"]
                                       for r_ in ranks),
                     "launcher": os.environ.get("SFTAMD_LAUNCHER", "external" if st.world_size > 1 else "none"),
                     "timeout_s": a.timeout_s, "hang_timeout_s": a.hang_timeout_s,
                     "rccl_info": rccl_dir is not None,
                     "rccl": mine.get("rccl"),
                     "p2p_transport": (mine.get("rccl") or {}).get("p2p_transport"),
                     "n_channels": (mine.get("rccl") or {}).get("n_channels"),
                     "n_channels_per_rank": [(r_.get("rccl") or {}).get("n_channels") for r_ in ranks],
                     "rccl_nranks_per_rank": [(r_.get("rccl") or {}).get("nranks") for r_ in ranks],
                     # every rank's communicator reported WORLD_SIZE ranks (None: no RCCL log, e.g. gloo)
                     "rccl_saw_all_ranks": (all((r_.get("rccl") or {}).get("nranks") == st.world_size for r_ in ranks)
                                            if rccl_dir is not None else None),
                     "link_probe": [[int(b), round(t * 1e3, 4)] for b, t in getattr(trainer, "link_points", [])],
                     "params_equal_across_ranks": len({_sum_key(r_["param_sum"]) for r_ in ranks}) == 1,
                     "warnings": dist_warn, "strict": strict},
            "optimizer_sharding": "zero1" if shard else "none",
            "bucket_plan": bucket_plan(trainer.engine),
            "comm_probe": probe,
            "comm_exposed_ms": max(r_["comm_exposed_ms"] for r_ in ranks),
            "per_rank": [{k: r_[k] for k in ("rank", "device", "ms_per_step", "peak_mem_gb", "comm_exposed_ms")}
                         for r_ in ranks],
        }
        if a.baseline_1gpu > 0:
            rec["scaling_efficiency"] = round(value / (st.world_size * a.baseline_1gpu), 4)
        print(json.dumps(rec), flush=True)
        if not math.isfinite(loss):
            # a non-finite loss makes the step faster (NaN / zero data toggles fewer bits, the clocks rise): the
            # throughput of such a run is not a measurement (profiles/r5_llama.md)
            print("[bench] WARNING: the loss is not finite; this run's throughput is void", file=sys.stderr, flush=True)
        for w in dist_warn:
            print(f"[bench] dist warning: {w}", file=sys.stderr, flush=True)
    if a.profile_steps:
        sync()
        prof = None
        if a.torch_profile:
            from torch.profiler import ProfilerActivity, profile
            prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True)
            prof.__enter__()
        for _ in range(a.profile_steps):
            step()
        trainer.optimizer.synchronize()
        sync()
        if prof is not None:
            prof.__exit__(None, None, None)
            if st.rank == 0:
                with open(a.torch_profile, "w") as f:
                    f.write(prof.key_averages(group_by_input_shape=True).table(
                        sort_by="self_device_time_total", row_limit=80, max_name_column_width=60,
                        max_shapes_column_width=90))
    if st.world_size > 1:
        barrier()
        dist.destroy_process_group()
    if strict and fatal:
        # the record above is printed (with dist.warnings) but the run fails loud: a scaling number measured over a
        # degraded transport must not pass as a healthy one
        sys.exit(3)
    if not math.isfinite(loss):
        # every rank holds the all-reduced loss: all exit non-zero, so a NaN run's throughput can never become a
        # BENCH / SCALE value (the record above carries loss_finite: false for the post-mortem)
        sys.exit(4)


def run_recipe(a):
    """``--recipe``: ``warmup + steps`` optimizer steps of the reference recipe through ``SFTTrainer.train()`` (the
    timed quantity is HF's: the whole train() wall time, evals included, like the reference's own metric)."""
    os.environ.setdefault("SFTAMD_HANG_TIMEOUT_S", str(a.hang_timeout_s))
    os.environ.setdefault("SFTAMD_RUN_DEADLINE_S", str(a.timeout_s))
    import torch

    from llm_fine_tune_distributed_amd.data.dataset import load_qa_parquet, train_test_split
    from llm_fine_tune_distributed_amd.data.prompts import format_prompt
    from llm_fine_tune_distributed_amd.data.tokenizer import load_tokenizer
    from llm_fine_tune_distributed_amd.models import build_model, get_config
    from llm_fine_tune_distributed_amd.parallel.process_group import cleanup_distributed, setup_distributed
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer

    st = setup_distributed(verbose=False, device="cpu" if a.device == "cpu" else None, timeout_s=a.hang_timeout_s + 60)
    on_gpu = st.device.type == "cuda"
    if on_gpu and a.tunableop != "off" and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ:
        from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(tune=(a.tunableop == "tune"), verbose=st.is_main)
    rows = load_qa_parquet(a.dataset)
    train_rows, val_rows = train_test_split(rows, test_size=0.1, seed=42)
    train_rows = [format_prompt(r) for r in train_rows]
    val_rows = [format_prompt(r) for r in val_rows]
    cfg = get_config(a.model)
    model = build_model(cfg, device=st.device, dtype=torch.bfloat16, seed=0)
    micro = 8 if a.micro_batch == 16 else a.micro_batch  # the recipe's own split: 8 x GA 2 (README.md:69)
    ga = 2 if a.ga == 1 else a.ga
    total = a.warmup + a.steps
    args = SFTConfig(output_dir="/tmp/sftamd_bench_recipe", per_device_train_batch_size=micro,
                     per_device_eval_batch_size=a.eval_batch, gradient_accumulation_steps=ga,
                     learning_rate=5e-5 * st.world_size, max_grad_norm=1.0, max_steps=total, logging_steps=2,
                     logging_first_step=True, eval_strategy="steps", eval_steps=a.eval_steps, save_strategy="no",
                     bf16=True, gradient_checkpointing=False, max_length=1024, dataloader_drop_last=True,
                     jsonl_log=False, freeze_policy=a.freeze_policy, shard_optimizer_state=bool(a.zero),
                     dataset_cache=False, gemm_tuning=False, optimizer_overlap=_overlap_arg(a),
                     padding_free={"auto": None, "on": True, "off": False}[a.padding_free],
                     **({} if a.ga_merge_max_tokens is None else {"ga_merge_max_tokens": a.ga_merge_max_tokens}))
    trainer = SFTTrainer(model=model, args=args, train_dataset=train_rows, eval_dataset=val_rows,
                         processing_class=load_tokenizer(None))
    if on_gpu:
        torch.cuda.synchronize()
    out = trainer.train()
    m = out.metrics
    evals = [h for h in trainer.state.log_history if "eval_loss" in h]
    if st.is_main:
        samples_per_step = micro * ga * st.world_size
        rec = {
            "metric": "samples/sec SmolLM3-3B full SFT bf16, reference recipe (HF train_samples_per_second incl. evals)"
            if a.model == "smollm3-3b" and a.freeze_policy == "full" else f"samples/sec {a.model} recipe",
            "value": round(m["train_samples_per_second"], 3), "unit": "samples/s", "n_gpus": st.world_size,
            "steps": total, "warmup": 0, "ms_per_step": round(m["train_runtime"] / max(1, out.global_step) * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "reference data/qa_dataset.parquet (offline synthetic tokenizer), random-init weights",
            "config": {"model": {"smollm3-3b": "SmolLM3-3B"}.get(a.model, a.model), "freeze_policy": a.freeze_policy,
                       "global_batch": samples_per_step, "per_device_batch": micro,
                       "gradient_accumulation_steps": ga, "seq_len": "ragged <= 1024 (padded to 64)",
                       "parallelism": f"dp{st.world_size}", "eval_steps": a.eval_steps,
                       "per_device_eval_batch": a.eval_batch, "padding_free": bool(trainer.packed)},
            "train_pure_samples_per_second": round(m["train_pure_samples_per_second"], 3),
            "train_tokens_per_second": round(m["train_tokens_per_second"], 1),
            "train_mfu": round(m.get("train_mfu", 0.0), 4), "train_runtime_s": round(m["train_runtime"], 3),
            "eval_runtime_s": round(sum(h.get("eval_runtime", 0.0) for h in evals), 3), "n_evals": len(evals),
            "final_eval_loss": round(evals[-1]["eval_loss"], 4) if evals else None,
            "train_loss": round(out.training_loss, 4),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2) if on_gpu else 0.0,
        }
        print(json.dumps(rec), flush=True)
    cleanup_distributed()


def _overlap_arg(a):
    """SFTConfig.optimizer_overlap from --overlap / --no-overlap."""
    if a.no_overlap:
        return False
    return {"auto": "auto", "on": True, "off": False}[a.overlap]


def _sum_key(x: float):
    """param_sum as a set key: every NaN the same (a NaN run is caught by the loss check, not as a rank mismatch)."""
    return "nan" if math.isnan(x) else x


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, argv))
    if a.recipe:
        run_recipe(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
