"""``SFTTrainer``: the TRL/HF-style supervised fine-tuning loop on the MI355X-native engine.

Reference surface (``training.py:289-312``): ``SFTTrainer(model, args, train_dataset,
eval_dataset, callbacks).train()`` -> ``TrainOutput``; ``.save_model(dir)``. The loop
reproduces the HF ``Trainer._inner_training_loop`` semantics the reference depends on
(SURVEY.md §3.2, T6):

* gradient accumulation over ``gradient_accumulation_steps`` micro-batches, gradient
  synchronisation only on the last one (``DDPEngine.no_sync``);
* loss normalisation by the GLOBAL number of non-ignored label tokens of the optimizer step
  (``num_items_in_batch`` summed over GA micro-batches and ranks): every micro-batch's loss is
  ``sum_token_CE / N_global`` and bucket all-reduces SUM, which equals HF's
  ``loss * world_size`` + averaging DDP;
* clip to ``max_grad_norm`` then AdamW then LR schedule step; logs ``loss, grad_norm,
  learning_rate, epoch`` (+ TRL's ``mean_token_accuracy, entropy, num_tokens``) every
  ``logging_steps``; eval every ``eval_steps`` with best-``eval_loss`` tracking; checkpoints
  every ``save_steps`` with rotation and ``resume_from_checkpoint``;
* end-of-train metrics ``train_runtime, train_samples_per_second, train_steps_per_second,
  total_flos, train_loss`` (HF definitions: wall time includes eval) plus pure-training
  samples/s, tokens/s and MFU.
"""
from __future__ import annotations

import contextlib
import math
import os
import random
import time
from typing import Any, Dict, List, NamedTuple, Optional, Sequence

import numpy as np
import torch

from ..data.collator import DataLoader, DistributedBatchSampler, SFTCollator
from ..data.dataset import TokenizedDataset, cached_tokenize
from .. import ops
from ..models import CausalLM, apply_freeze_policy, build_model, get_config
from ..models.lora import LoRAConfig
from ..parallel.ddp import DDPEngine
from ..parallel.process_group import all_reduce_sum_, all_reduce_sum_async, barrier, setup_distributed
from . import checkpoint as ckpt
from .callbacks import (AimCallback, CallbackHandler, JSONLLoggerCallback, PrinterCallback, TrainerCallback,
                        TrainerControl, TrainerState)
from .config import SFTConfig
from .optim import FlatAdamW, LRScheduler, ShardedAdamW, get_schedule
from ..utils.faults import maybe_inject

PEAK_BF16_FLOPS = 2.5e15  # MI355X dense bf16 (vendor figure; AMD's 5 PF headline includes 2:1 sparsity)


class TrainOutput(NamedTuple):
    global_step: int
    training_loss: float
    metrics: Dict[str, float]


def set_seed(seed: int):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


class SFTTrainer:
    def __init__(self, model=None, args: Optional[SFTConfig] = None, train_dataset=None, eval_dataset=None,
                 processing_class=None, tokenizer=None, callbacks: Optional[Sequence[TrainerCallback]] = None,
                 data_collator: Optional[SFTCollator] = None, peft_config: Optional[LoRAConfig] = None,
                 model_init_seed: int = 0):
        self.args = args = args or SFTConfig()
        self.dist = setup_distributed(timeout_s=args.ddp_timeout, verbose=False)
        # context parallelism: consecutive ranks form CP groups that share each batch, sequence-sharded
        # (ring attention); data parallelism runs across the groups
        self.cp_size = int(getattr(args, "context_parallel_size", 1) or 1)
        self.cp_group, self.cp_rank, self.dp_rank, self.dp_size = None, 0, self.dist.rank, self.dist.world_size
        if self.cp_size > 1:
            from ..parallel.context_parallel import new_groups
            if args.packing:
                raise ValueError("context_parallel_size > 1 needs padded batches (packing=False)")
            self.cp_group, self.cp_rank, self.dp_rank, self.dp_size = new_groups(
                self.dist.world_size, self.dist.rank, self.cp_size)
        set_seed(args.seed)
        dev = self.dist.device
        pf = getattr(args, "padding_free", None)
        self.packed = bool(args.packing) or (bool(pf) if pf is not None else (dev.type == "cuda" and self.cp_size == 1))
        if self.packed and self.cp_size > 1:
            raise ValueError("context_parallel_size > 1 needs padded batches (packing / padding_free off)")
        if (args.gemm_tuning and dev.type == "cuda" and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ
                and not torch.cuda.tunable.is_enabled()):  # a caller's own TunableOp setup (e.g. tuning) wins
            from ..utils.gemm_tuning import enable_tuned_gemms
            enable_tuned_gemms()
        # ------------------------------------------------------------ model
        if isinstance(model, str):
            if os.path.isdir(model) and any(f.endswith(".safetensors") for f in os.listdir(model)):
                model = ckpt.from_pretrained(model, device=dev, dtype=torch.bfloat16)
            else:
                model = build_model(get_config(model), device=dev, dtype=torch.bfloat16, seed=model_init_seed)
        assert isinstance(model, CausalLM), "SFTTrainer expects a CausalLM (or a preset name / HF dir)"
        if next(model.parameters()).device != dev:
            model.to(dev)
            model.inv_freq = model.inv_freq.to(dev)
        self.model = model
        if peft_config is not None or args.freeze_policy != "full":
            lc = peft_config or LoRAConfig(r=args.lora_r, lora_alpha=args.lora_alpha, lora_dropout=args.lora_dropout,
                                           **({"target_modules": args.lora_target_modules} if args.lora_target_modules else {}))
            policy = "lora" if peft_config is not None else args.freeze_policy
            apply_freeze_policy(model, policy, n_last=args.freeze_last_n_layers, lora_config=lc)
        if args.gradient_checkpointing:
            model.gradient_checkpointing_enable()
        if self.cp_size > 1:
            model.enable_context_parallel(self.cp_group, args.context_parallel_layout)
        self.trainable_params = model.num_parameters(trainable_only=True)
        self.total_params = model.num_parameters()
        # ------------------------------------------------------------ data
        self.tokenizer = processing_class or tokenizer
        if self.tokenizer is None and (self._needs_tokenizer(train_dataset) or self._needs_tokenizer(eval_dataset)):
            self.tokenizer = self._main_first_tokenizer()
        self.train_dataset = self._prepare(train_dataset, args.max_train_samples)
        self.eval_dataset = self._prepare(eval_dataset, args.max_eval_samples)
        pad_id = self.tokenizer.pad_token_id if self.tokenizer is not None else (model.config.pad_token_id or 0)
        self._pad_id = pad_id
        pad_mult = args.pad_to_multiple_of
        if pad_mult is None and dev.type == "cuda":
            pad_mult = 256 if self.packed else 64
        # explicit packing: at most per_device_train_batch_size x max_length tokens per batch; padding-free: the whole
        # batch, however long (every sample of the padded batch, none dropped)
        self.collator = data_collator or SFTCollator(pad_id, pad_mult, args.max_length, self.packed,
                                                     args.per_device_train_batch_size * (args.max_length or 1024)
                                                     if args.packing else None)
        # ------------------------------------------------------------ engine + optimizer
        shard = bool(args.shard_optimizer_state) and self.dist.world_size > 1
        link, self.link_points = None, []
        if self.dist.world_size > 1 and not args.ddp_bucket_cap_mb and args.ddp_link_probe:
            # measured collective cost -> bucket cap (every rank fits the same max-over-ranks timings)
            from ..parallel.ddp import fit_link, measure_link
            self.link_points = measure_link(self.dist.world_size, dev)
            # None (a clamped fit: noise) -> the modelled 30 us / 100 GB/s plan, recorded as plan_source "model"
            link = fit_link(self.link_points, self.dist.world_size, strict=True)
        self.engine = DDPEngine(model, self.dist.world_size, self.dist.rank,
                                bucket_cap_mb=args.ddp_bucket_cap_mb,  # None: xGMI plan (plan_bucket_mb)
                                first_bucket_mb=args.ddp_first_bucket_mb,
                                broadcast_params=args.ddp_broadcast_params, shard=shard, link=link)
        if self.engine.tied_sparse:
            self.engine.sparse_cap = self._sparse_cap()
        opt_cls = ShardedAdamW if shard else FlatAdamW
        self.optimizer = opt_cls(self.engine, lr=args.learning_rate, betas=(args.adam_beta1, args.adam_beta2),
                                   eps=args.adam_epsilon, weight_decay=args.weight_decay,
                                   master_weights=args.master_weights,
                                   stochastic_rounding=args.stochastic_rounding,
                                   state_dtype=args.optim_state_dtype)
        overlap = args.optimizer_overlap
        if overlap == "auto":
            overlap = self.dist.world_size > 1
        if overlap and dev.type == "cuda":
            self.optimizer.enable_overlap(model)
        self.scheduler: Optional[LRScheduler] = None
        # ------------------------------------------------------------ callbacks / state
        self.state = TrainerState(is_world_process_zero=self.dist.is_main)
        self.control = TrainerControl()
        cbs = list(callbacks or [])
        if args.jsonl_log and self.dist.is_main:
            cbs.append(JSONLLoggerCallback(os.path.join(args.output_dir, "metrics.jsonl")))
        cbs.append(PrinterCallback())
        self.callback_handler = CallbackHandler(cbs)
        self._timers: Dict[str, float] = {"eval": 0.0}
        from ..utils.profiling import StepTimer
        self.phase_timer = StepTimer(enabled=dev.type == "cuda") if args.log_step_phases else None
        self._log_count = 0
        # per-rank heartbeat (step, phase, last gradient bucket issued): the launcher's hang detector reads it, the
        # watchdog thread (SFTAMD_HANG_TIMEOUT_S / SFTAMD_RUN_DEADLINE_S) ends a stuck rank with exit code 124
        from ..utils import heartbeat as hb
        eng = self.engine
        info = lambda: {"bucket": eng.last_launched, "buckets": len(eng.buckets)}  # noqa: E731
        self.heartbeat = hb.get() or hb.install(hb.Heartbeat(self.dist.rank, info=info))
        if self.heartbeat.info is None:  # a caller's heartbeat (bench.py): add this engine's bucket position
            self.heartbeat.info = info
        self._hb_step = 0

    def _sparse_cap(self) -> int:
        """Most tokens one synchronising pass can hold, identical on every rank: the sparse tied-embedding exchange
        gathers that many rows without a device sync. Derived from the collator in use and the training data it
        will see (``SFTCollator.max_batch_tokens``: the bound holds by construction, so no rank can overflow it while
        the others wait in the gather). 0 (= every rank measures the pass with a MAX all-reduce) for a custom
        collator, an unknown dataset, or a bound so large the dense path is as cheap."""
        a = self.args
        if type(self.collator) is not SFTCollator or not isinstance(self.train_dataset, TokenizedDataset):
            return 0
        B = a.per_device_train_batch_size
        per_pass = self.collator.max_batch_tokens(self.train_dataset, B)
        if per_pass <= 0:
            return 0
        if self.cp_size > 1:  # shard_batch pads T to 2 cp (zig-zag) / cp and hands each rank B x Tp / cp tokens
            unit = 2 * self.cp_size if a.context_parallel_layout == "zigzag" else self.cp_size
            T = per_pass // B
            per_pass = B * (-(-T // unit) * unit) // self.cp_size
        elif a.gradient_accumulation_steps > 1 and getattr(a, "ga_merge_max_tokens", 0):
            per_pass = max(per_pass, int(a.ga_merge_max_tokens))  # a merged pass holds at most this many
        V = self.model.config.vocab_size
        return per_pass if per_pass * self.dist.world_size < V else 0

    # ------------------------------------------------------------------ data helpers
    @staticmethod
    def _needs_tokenizer(ds) -> bool:
        return ds is not None and not isinstance(ds, TokenizedDataset)

    def _cache_dir(self) -> Optional[str]:
        a = self.args
        if not a.dataset_cache:
            return None
        return a.dataset_cache if isinstance(a.dataset_cache, str) else os.path.join(a.output_dir, ".sftamd_cache")

    def _main_first_tokenizer(self):
        """Offline synthetic tokenizer, trained ONCE: rank 0 trains and saves it, the others load it."""
        from ..data.tokenizer import load_tokenizer
        cache = self._cache_dir()
        if cache is None or self.dist.world_size == 1:
            return load_tokenizer()
        tdir = os.path.join(cache, "tokenizer")
        if self.dist.is_main:
            tk = load_tokenizer()
            tmp = f"{tdir}.tmp{os.getpid()}"
            tk.save_pretrained(tmp)
            if os.path.isdir(tdir):
                import shutil
                shutil.rmtree(tdir, ignore_errors=True)
            os.replace(tmp, tdir)
        barrier()
        return tk if self.dist.is_main else load_tokenizer(tdir)

    def _prepare(self, ds, limit):
        if ds is None:
            return None
        if isinstance(ds, TokenizedDataset):
            return ds
        rows = list(ds) if not isinstance(ds, list) else ds
        if limit:
            rows = rows[:limit]
        return cached_tokenize(rows, self.tokenizer, self._cache_dir(), is_main=self.dist.is_main,
                               barrier=barrier if self.dist.world_size > 1 else None, max_length=self.args.max_length,
                               assistant_only_loss=self.args.assistant_only_loss,
                               text_field=self.args.dataset_text_field)

    def get_train_dataloader(self) -> DataLoader:
        a = self.args
        s = DistributedBatchSampler(len(self.train_dataset), a.per_device_train_batch_size, self.dp_size,
                                    self.dp_rank, shuffle=True, seed=a.data_seed or a.seed,
                                    drop_last=a.dataloader_drop_last)
        return DataLoader(self.train_dataset, self.collator, s, self.dist.device, a.dataloader_pin_memory,
                          a.prefetch_batches)

    def get_eval_dataloader(self) -> DataLoader:
        a = self.args
        s = DistributedBatchSampler(len(self.eval_dataset), a.per_device_eval_batch_size, self.dp_size,
                                    self.dp_rank, shuffle=False, drop_last=a.dataloader_drop_last)
        return DataLoader(self.eval_dataset, self.collator, s, self.dist.device, a.dataloader_pin_memory,
                          a.prefetch_batches)

    # ------------------------------------------------------------------ core step
    @staticmethod
    def _model_inputs(b: Dict) -> Dict:
        kw = {"input_ids": b["input_ids"], "labels": b["labels"]}
        if "cu_seqlens" in b:
            kw.update(cu_seqlens=b["cu_seqlens"], position_ids=b["position_ids"], max_seqlen=b["max_seqlen"],
                      shift_labels=not b.get("shifted", False))
        elif "position_ids" in b:  # context-parallel chunk: global positions, labels shifted before sharding
            kw.update(position_ids=b["position_ids"], shift_labels=not b.get("shifted", False))
        return kw

    def _cp_shard(self, b: Dict) -> Dict:
        if self.cp_size == 1:
            return b
        from ..parallel.context_parallel import shard_batch
        return shard_batch(b, self.cp_rank, self.cp_size, self._pad_id, self.args.context_parallel_layout)

    def global_num_items(self, micro: List[Dict]):
        """Global count of loss tokens of this optimizer step (TRL ``num_items_in_batch``).

        With more than one rank the 1-float all-reduce is issued asynchronously and handed to the model
        as a ``PendingCount``, resolved only where the loss needs it (after the last decoder layer).
        Under ZeRO-1 the previous step's parameter all-gathers are still queued on the same RCCL
        communicator: a blocking all-reduce here would make the compute stream wait for ALL of them
        before the first layer, serialising the gather that is meant to run under the forward.
        """
        if all(torch.is_tensor(b.get("num_items_t")) for b in micro):
            n = micro[0]["num_items_t"].to(self.dist.device, non_blocking=True).clone()
            for b in micro[1:]:
                n += b["num_items_t"].to(self.dist.device, non_blocking=True)
        else:
            n = torch.tensor([float(sum(b["num_items"] for b in micro))], device=self.dist.device)
        if self.args.average_tokens_across_devices:
            return all_reduce_sum_async(n)
        # per-rank normalisation (HF: local mean per DATA-PARALLEL rank, DDP then AVERAGES the gradients): the buckets
        # are SUM-reduced here, so the local count is scaled by the data-parallel size. Under context parallelism a
        # DP rank's batch is split over its CP group: its local count is the CP group's sum, not this chunk's
        if self.cp_size > 1:
            return all_reduce_sum_async(n, group=self.cp_group, scale=float(self.dp_size))
        return n.clamp(min=1.0) * self.dist.world_size

    def _phase(self, name: str, host: bool = False):
        """Step-phase timing + roctx range (``log_step_phases``); a no-op otherwise."""
        t = self.phase_timer
        return t.phase(name, host=host) if t is not None else contextlib.nullcontext()

    def _merge_micro(self, micro: List[Dict]) -> List[Dict]:
        """Run the step's GA micro-batches as one pass when they fit ``ga_merge_max_tokens`` (see SFTConfig):
        padded batches are re-padded to the longest and stacked, packed (varlen) batches are concatenated with
        shifted ``cu_seqlens``. The per-batch scalars (token / sample / label counts) are summed."""
        cap = int(getattr(self.args, "ga_merge_max_tokens", 0) or 0)
        if len(micro) < 2 or cap <= 0 or self.cp_size > 1:
            return micro
        packed = "cu_seqlens" in micro[0]
        if any(("cu_seqlens" in b) != packed for b in micro):
            return micro
        total = sum(b["input_ids"].numel() for b in micro) if packed else \
            sum(b["input_ids"].shape[0] for b in micro) * max(b["input_ids"].shape[1] for b in micro)
        if total > cap:
            return micro
        out = {k: sum(b[k] for b in micro) for k in ("num_items", "num_samples", "num_tokens")}
        if all(torch.is_tensor(b.get("num_items_t")) for b in micro):
            out["num_items_t"] = torch.stack([b["num_items_t"] for b in micro]).sum(0)
        if packed:
            cus, off = [micro[0]["cu_seqlens"]], micro[0]["cu_seqlens"][-1:]
            for b in micro[1:]:
                cus.append(b["cu_seqlens"][1:] + off)
                off = off + b["cu_seqlens"][-1:]
            out.update(input_ids=torch.cat([b["input_ids"] for b in micro]),
                       labels=torch.cat([b["labels"] for b in micro]), cu_seqlens=torch.cat(cus),
                       position_ids=torch.cat([b["position_ids"] for b in micro]),
                       max_seqlen=max(b["max_seqlen"] for b in micro), shifted=micro[0].get("shifted", False))
        else:
            T = max(b["input_ids"].shape[1] for b in micro)
            F = torch.nn.functional
            out.update(input_ids=torch.cat([F.pad(b["input_ids"], (0, T - b["input_ids"].shape[1]), value=self._pad_id)
                                            for b in micro]),
                       labels=torch.cat([F.pad(b["labels"], (0, T - b["labels"].shape[1]), value=-100) for b in micro]))
        return [out]

    def optimizer_step(self, micro: List[Dict], lr: float) -> Dict[str, torch.Tensor]:
        """One optimizer step over ``micro`` (GA micro-batches). Returns device-side sums:
        loss (this rank's share of the global mean), correct, entropy_sum, valid tokens."""
        return self._optimizer_step(micro, lr)

    def _optimizer_step(self, micro: List[Dict], lr: float) -> Dict[str, torch.Tensor]:
        model, eng = self.model, self.engine
        model.train()
        self._hb_step += 1
        beat = self.heartbeat.beat
        micro = self._merge_micro([self._cp_shard(b) for b in micro])
        n_items = self.global_num_items(micro)
        acc = torch.zeros(4, device=self.dist.device)  # loss, correct, entropy_sum, valid
        for i, b in enumerate(micro):
            sync = i == len(micro) - 1
            ctx = contextlib.nullcontext() if sync else eng.no_sync()
            with ctx:
                eng.prepare_backward()
                beat(self._hb_step, "fwd", micro=i)
                with self._phase("fwd"):
                    out = model(**self._model_inputs(b), num_items_in_batch=n_items)
                beat(self._hb_step, "bwd", micro=i)
                with self._phase("bwd"):
                    out.loss.backward()
            acc[0] += out.loss.detach()
            acc[1:] += out.metrics
        beat(self._hb_step, "comm_wait")
        with self._phase("comm_wait"):
            eng.finish_backward()
        beat(self._hb_step, "optim")
        with self._phase("optim"):
            norm = self.optimizer.step(lr=lr, max_grad_norm=self.args.max_grad_norm)
        eng.zero_grad()
        return {"acc": acc, "grad_norm": norm}

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, eval_dataset=None, metric_key_prefix: str = "eval") -> Dict[str, float]:
        if eval_dataset is not None:
            self.eval_dataset = self._prepare(eval_dataset, self.args.max_eval_samples)
        if self.eval_dataset is None:
            return {}
        t0 = time.time()
        self.optimizer.synchronize()
        self.model.eval()
        acc = torch.zeros(5, device=self.dist.device)  # loss_sum, correct, entropy_sum, valid, samples
        loader = self.get_eval_dataloader()
        beat = self.heartbeat.beat
        for b in loader:
            beat(self._hb_step, "eval")
            b = self._cp_shard(b)
            out = self.model(**self._model_inputs(b), num_items_in_batch=1.0)
            acc[0] += out.loss
            acc[1:4] += out.metrics
            acc[4] += b["num_samples"] if self.cp_rank == 0 else 0  # a CP group shares its samples
        all_reduce_sum_(acc)
        vals = acc.tolist()
        self.model.train()
        rt = time.time() - t0
        valid = max(vals[3], 1.0)
        nb = len(loader) * self.dp_size
        m = {f"{metric_key_prefix}_loss": vals[0] / valid, f"{metric_key_prefix}_runtime": rt,
             f"{metric_key_prefix}_samples_per_second": vals[4] / max(rt, 1e-9),
             f"{metric_key_prefix}_steps_per_second": nb / max(rt, 1e-9),
             f"{metric_key_prefix}_mean_token_accuracy": vals[1] / valid,
             f"{metric_key_prefix}_entropy": vals[2] / valid, f"{metric_key_prefix}_num_tokens": vals[3],
             "epoch": self.state.epoch}
        self._timers["eval"] += rt
        self.callback_handler.call("on_evaluate", self.args, self.state, self.control, metrics=m)
        self.log(m)
        return m

    # ------------------------------------------------------------------ logging / saving
    def log(self, logs: Dict[str, Any]):
        logs = dict(logs)
        logs.setdefault("step", self.state.global_step)
        self.state.log_history.append(dict(logs))
        self.control = self.callback_handler.call("on_log", self.args, self.state, self.control, logs=logs)

    def _save_checkpoint(self):
        with self.heartbeat.hold("ckpt_save", step=self._hb_step):  # rank 0 writes while the others wait
            return self._save_checkpoint_impl()

    def _save_checkpoint_impl(self):
        self.optimizer.synchronize()
        a = self.args
        path = os.path.join(a.output_dir, f"checkpoint-{self.state.global_step}")
        # EVERY rank takes part: under ZeRO-1 the shards are gathered onto rank 0 (a collective that would deadlock if
        # only rank 0 entered it while the others wait in the barrier); no other rank builds a full host copy
        osd = self.optimizer.state_dict(dst=0)
        barrier()
        ckpt.save_rng(path, self.dist.rank)
        ckpt.save_checkpoint(path, self.model, self.optimizer, self.scheduler, self.state, a, self.dist.rank,
                             tokenizer=self.tokenizer, optimizer_state=osd if self.dist.is_main else {})
        del osd
        barrier()
        if self.dist.is_main:
            ckpt.rotate_checkpoints(a.output_dir, a.save_total_limit, self.state.best_model_checkpoint)
        barrier()
        self.callback_handler.call("on_save", a, self.state, self.control)
        return path

    def save_model(self, output_dir: Optional[str] = None, merge_lora: bool = False):
        """Rank 0 writes the HF directory; every rank waits. ``merge_lora`` folds LoRA adapters into the
        saved weights (export for plain HF / llama.cpp consumers) instead of writing them separately."""
        output_dir = output_dir or self.args.output_dir
        with self.heartbeat.hold("save_model", step=self._hb_step):
            self.optimizer.synchronize()
            if self.dist.is_main:
                ckpt.save_pretrained(self.model, output_dir, tokenizer=self.tokenizer, merge_lora=merge_lora)
            barrier()

    def _update_best(self, metrics: Dict[str, float], ckpt_path: Optional[str]):
        key = self.args.metric_for_best_model or "eval_loss"
        if not key.startswith("eval_"):
            key = "eval_" + key
        if key not in metrics:
            return
        v = metrics[key]
        gib = self.args.greater_is_better
        if gib is None:
            gib = not key.endswith("loss")
        b = self.state.best_metric
        if b is None or (v > b if gib else v < b):
            self.state.best_metric = v
            if ckpt_path:
                self.state.best_model_checkpoint = ckpt_path

    # ------------------------------------------------------------------ train
    def train(self, resume_from_checkpoint: Optional[str] = None) -> TrainOutput:
        """The training loop; the hang watchdog is armed only while it runs (slow phases inside it — checkpoint
        load / save, the first step — under ``Heartbeat.hold``)."""
        self.heartbeat.resume()
        try:
            return self._train(resume_from_checkpoint)
        finally:
            self.heartbeat.pause()

    def _train(self, resume_from_checkpoint: Optional[str] = None) -> TrainOutput:
        a = self.args
        loader = self.get_train_dataloader()
        ga = max(1, a.gradient_accumulation_steps)
        nb = len(loader)
        steps_per_epoch = max(1, nb // ga + int(nb % ga > 0))
        max_steps = a.max_steps if a.max_steps and a.max_steps > 0 else math.ceil(a.num_train_epochs * steps_per_epoch)
        warm = a.warmup_steps or int(math.ceil(a.warmup_ratio * max_steps))
        self.scheduler = LRScheduler(self.optimizer, get_schedule(a.lr_scheduler_type, max_steps, warm,
                                                                  **a.lr_scheduler_kwargs))
        self.state.max_steps = max_steps
        self.state.num_train_epochs = math.ceil(max_steps / steps_per_epoch)
        self.state.train_batch_size = a.per_device_train_batch_size
        start_epoch, skip_batches = 0, 0
        resume = resume_from_checkpoint or a.resume_from_checkpoint
        if resume:
            if resume is True or resume == "auto":
                resume = ckpt.latest_checkpoint(a.output_dir)
            if resume:
                with self.heartbeat.hold("ckpt_load"):
                    st, _ = ckpt.load_checkpoint(resume, self.model, self.optimizer, self.scheduler, self.dist.rank)
                st.is_world_process_zero = self.dist.is_main
                self.state = st
                start_epoch = self.state.global_step // steps_per_epoch
                skip_batches = (self.state.global_step % steps_per_epoch) * ga
                if self.dist.is_main:
                    print(f"[trainer] resumed from {resume} at step {self.state.global_step}", flush=True)
        if self.dist.is_main:
            print(f"[trainer] world={self.dist.world_size} device={self.dist.device} trainable="
                  f"{self.trainable_params:,}/{self.total_params:,} "
                  f"({100.0 * self.trainable_params / max(1, self.total_params):.2f}%) steps={max_steps} "
                  f"ga={ga} micro={a.per_device_train_batch_size}", flush=True)
        self.control = self.callback_handler.call("on_train_begin", a, self.state, self.control)
        eval_every = a.resolved_eval_steps()
        log_every = max(1, int(a.logging_steps)) if a.logging_steps else 0
        save_every = int(a.save_steps) if a.save_strategy == "steps" and a.save_steps else 0
        cfg = self.model.config
        run_acc = torch.zeros(4, device=self.dist.device)
        steps_since_log = 0
        total_loss = torch.zeros(1, device=self.dist.device)
        samples = tokens = 0
        flops = 0.0
        t_start = time.time()
        self._timers["eval"] = 0.0
        last_norm = None
        done = self.state.global_step >= max_steps
        start_step = self.state.global_step  # train_loss averages the steps run by THIS call
        for epoch in range(start_epoch, self.state.num_train_epochs):
            if done:
                break
            loader.set_epoch(epoch)
            self.control = self.callback_handler.call("on_epoch_begin", a, self.state, self.control)
            it = loader.iter(skip=skip_batches if epoch == start_epoch else 0)
            step_in_epoch = (skip_batches // ga) if epoch == start_epoch else 0
            while True:
                micro = []
                with self._phase("data", host=True):
                    for _ in range(ga):
                        try:
                            micro.append(next(it))
                        except StopIteration:
                            break
                if not micro:
                    break
                self.control = self.callback_handler.call("on_step_begin", a, self.state, self.control)
                lr = self.scheduler.get_lr()
                if self.state.global_step == start_step:  # first step: GEMM tuning / warm-up may take a while
                    with self.heartbeat.hold("first_step", step=self._hb_step + 1):
                        r = self.optimizer_step(micro, lr)
                else:
                    r = self.optimizer_step(micro, lr)
                self.scheduler.step()
                run_acc += r["acc"]
                total_loss += r["acc"][0]
                last_norm = r["grad_norm"]
                steps_since_log += 1
                n_s = sum(b["num_samples"] for b in micro)
                n_t = sum(b["num_tokens"] for b in micro)
                samples += n_s * self.dp_size  # a context-parallel group shares its samples
                tokens += n_t * self.dp_size
                T = max(b["input_ids"].shape[-1] for b in micro)
                flops += cfg.flops_per_token(T, training=True, recompute=a.gradient_checkpointing) * n_t * \
                    self.dp_size
                self.state.global_step += 1
                step_in_epoch += 1
                self.state.epoch = epoch + step_in_epoch / steps_per_epoch
                self.state.samples_seen += n_s * self.dp_size
                self.state.tokens_seen += n_t * self.dp_size
                self.state.total_flos += 6.0 * self.trainable_params * n_t * self.dp_size
                self.control = self.callback_handler.call("on_step_end", a, self.state, self.control)
                gs = self.state.global_step
                maybe_inject(self.dist.rank, gs)
                if log_every and (gs % log_every == 0 or (gs == 1 and a.logging_first_step)):
                    red = run_acc.clone()
                    all_reduce_sum_(red)
                    v = red.tolist()
                    valid = max(v[3], 1.0)
                    logs = {"loss": v[0] / steps_since_log, "grad_norm": float(last_norm),
                            "learning_rate": self.scheduler.get_lr(), "epoch": round(self.state.epoch, 4),
                            "mean_token_accuracy": v[1] / valid, "entropy": v[2] / valid,
                            "num_tokens": float(self.state.tokens_seen)}
                    if self.dist.device.type == "cuda":
                        logs["hbm_peak_gb"] = round(torch.cuda.max_memory_allocated(self.dist.device) / 1e9, 3)
                        if self.dist.world_size > 1:
                            logs["comm_exposed_ms"] = round(self.engine.comm_exposed_ms(), 3)
                    if self.phase_timer is not None:  # mean per optimizer step since the last log
                        for k, v in self.phase_timer.summary().items():
                            logs[f"{k}_ms"] = round(v / steps_since_log, 3)
                    self._log_count += 1
                    if a.log_system_metrics_every and self._log_count % a.log_system_metrics_every == 0 \
                            and self.dist.is_main:
                        from ..utils.telemetry import system_log_entries
                        logs.update(system_log_entries())
                    self.log(logs)
                    if not math.isfinite(logs["loss"]):
                        # (the loss was read for the log anyway: the check adds no host sync)
                        self.state.nonfinite_loss_steps.append(gs)
                        self.heartbeat.beat(gs, "nonfinite_loss", loss=str(logs["loss"]))
                        if self.dist.is_main:
                            print(f"[trainer] WARNING: non-finite loss {logs['loss']} at step {gs}", flush=True)
                        if a.stop_on_nonfinite_loss:
                            self.control.should_training_stop = True
                    run_acc.zero_()
                    steps_since_log = 0
                if a.ddp_check_sync_every and gs % a.ddp_check_sync_every == 0:
                    self.optimizer.synchronize()  # pending (overlapped) updates / gathers land first
                    self.engine.assert_in_sync()
                metrics = None
                if eval_every and eval_every > 0 and gs % eval_every == 0 and self.eval_dataset is not None:
                    metrics = self.evaluate()
                ck = None
                if save_every and gs % save_every == 0:
                    ck = self._save_checkpoint()
                if metrics:
                    self._update_best(metrics, ck)
                if gs >= max_steps or self.control.should_training_stop:
                    done = True
                    break
            if eval_every == -1 and self.eval_dataset is not None:
                m = self.evaluate()
                self._update_best(m, None)
            self.control = self.callback_handler.call("on_epoch_end", a, self.state, self.control)
        self.optimizer.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        runtime = time.time() - t_start
        tl = total_loss.clone()
        all_reduce_sum_(tl)
        steps_run = self.state.global_step - start_step
        train_loss = tl.item() / max(1, steps_run)  # (HF divides by global_step, under-reporting after a resume)
        pure = max(runtime - self._timers["eval"], 1e-9)
        metrics = {"train_runtime": runtime, "train_samples_per_second": samples / max(runtime, 1e-9),
                   "train_steps_per_second": self.state.global_step / max(runtime, 1e-9),
                   "total_flos": self.state.total_flos, "train_loss": train_loss, "epoch": self.state.epoch,
                   "train_pure_samples_per_second": samples / pure, "train_tokens_per_second": tokens / pure,
                   "train_mfu": flops / pure / (PEAK_BF16_FLOPS * self.dist.world_size)
                   if self.dist.device.type == "cuda" else 0.0}
        if a.load_best_model_at_end and self.state.best_model_checkpoint:
            self.heartbeat.pause()  # host-side load: nothing beats
            sd = ckpt.load_state_dict(self.state.best_model_checkpoint, device="cpu")
            with torch.no_grad():
                self.model.load_hf_state_dict({k: v.to(torch.bfloat16) for k, v in sd.items()}, strict=False)
        self.log(metrics)
        self.control = self.callback_handler.call("on_train_end", a, self.state, self.control)
        return TrainOutput(self.state.global_step, train_loss, metrics)
