"""Flat AdamW + LR schedules (reference T3/T4/T5).

The reference runs HF's default ``adamw_torch(_fused)`` over bf16 parameters with
``lr = LEARNING_RATE * WORLD_SIZE`` (training.py:263), betas (0.9, 0.999), eps 1e-8, wd 0, and
``lr_scheduler_type="linear"`` (decay to 0, no warmup). Here the update is ONE fused HIP kernel
per weight-decay region over the DDP engine's flat buffers, with an fp32 master copy and fp32
moments by default (``master_weights=False`` reproduces the reference's pure-bf16 parameter
update with fp32 moments). Gradient clipping (max_grad_norm) is a flat sum-of-squares kernel;
the clip coefficient never leaves the GPU.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional

import torch

from .. import ops


class FlatAdamW:
    def __init__(self, engine, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 master_weights: bool = True, stochastic_rounding: bool = True, state_dtype=torch.float32):
        """``state_dtype`` = dtype of exp_avg / exp_avg_sq: fp32 (default) or bf16 — what torch's
        AdamW keeps for the reference's bf16 parameters (training.py:99) — stored with stochastic
        rounding (unbiased) when ``stochastic_rounding`` is on; 8 fewer HBM bytes per parameter."""
        self.engine = engine
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.master_weights = master_weights
        self.stochastic_rounding = stochastic_rounding and not master_weights
        self.step_count = 0
        n = engine.numel
        dev = engine.device
        if isinstance(state_dtype, str):
            state_dtype = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
                           "bfloat16": torch.bfloat16}[state_dtype]
        if state_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"optimizer state dtype must be fp32 or bf16, got {state_dtype}")
        self.state_dtype = state_dtype
        self.master = engine.param_flat.float() if master_weights else None
        self.exp_avg = torch.zeros(n, dtype=state_dtype, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=state_dtype, device=dev)
        self.last_grad_norm: Optional[torch.Tensor] = None
        self.overlap = False

    # ------------------------------------------------------------------ overlap with next forward
    def enable_overlap(self, model) -> bool:
        """Pipeline the update under the NEXT step's forward (MI355X: AdamW is HBM-bound, the
        forward GEMMs are MFMA-bound, so they co-run well). Updates are issued on a side stream in
        forward order (embedding, layer 0, ..., layer L-1, final norm/head), one event per group;
        forward pre-hooks make the compute stream wait only for the group it is about to read."""
        if not self.engine.param_flat.is_cuda:
            return False
        e = self.engine
        region_of = {}
        for s, t, decay in e.regions:
            region_of[(s, t)] = decay
        offs = {id(p): (o, n) for p, o, n, _ in e.layout}

        def ranges(params):
            rs = []
            for p in params:
                if id(p) not in offs:
                    continue
                o, n = offs[id(p)]
                n = (n + 63) // 64 * 64
                decay = next(d for (s, t), d in region_of.items() if s <= o < t)
                rs.append([o, o + n, decay])
            rs.sort()
            merged = []
            for r in rs:
                if merged and merged[-1][1] == r[0] and merged[-1][2] == r[2]:
                    merged[-1][1] = r[1]
                else:
                    merged.append(r)
            return merged

        inner = model.model
        seen = set()
        groups = []

        def add(mods_params):
            ps = [p for p in mods_params if id(p) not in seen]
            for p in ps:
                seen.add(id(p))
            groups.append(ranges(ps))

        add([inner.embed_tokens])
        for layer in inner.layers:
            add(list(layer.parameters()))
        add(list(inner.norm.parameters()) + ([model.lm_head] if model.lm_head is not None else []))
        rest = [p for p, _, _, _ in e.layout if id(p) not in seen]
        if rest:
            groups[-1] += ranges(rest)
        self._groups = groups
        self._events = [torch.cuda.Event() for _ in groups]
        self._stream = torch.cuda.Stream(device=e.device)
        self._pending = False
        self._hooks = []

        def waiter(i):
            def hook(*_a, **_k):
                if self._pending:
                    torch.cuda.current_stream().wait_event(self._events[i])
            return hook

        self._hooks.append(model.register_forward_pre_hook(waiter(0)))
        for i, layer in enumerate(inner.layers):
            self._hooks.append(layer.register_forward_pre_hook(waiter(i + 1)))
        self._hooks.append(inner.layers[-1].register_forward_hook(waiter(len(groups) - 1)))
        self.overlap = True
        return True

    def synchronize(self):
        """Make the current stream wait for every pending update (before eval / save / logging)."""
        if getattr(self, "_pending", False):
            cs = torch.cuda.current_stream()
            for ev in self._events:
                cs.wait_event(ev)
            self._pending = False

    @torch.no_grad()
    def step(self, lr: Optional[float] = None, max_grad_norm: Optional[float] = None):
        lr = self.lr if lr is None else lr
        self.step_count += 1
        e = self.engine
        self.synchronize()
        norm, coef = ops.grad_norm_flat([e.grad_flat], max_grad_norm if max_grad_norm else 0.0)
        self.last_grad_norm = norm
        b1, b2 = self.betas

        def upd(s, t, decay):
            ops.adamw_flat_(e.param_flat[s:t], e.grad_flat[s:t], None if self.master is None else self.master[s:t],
                            self.exp_avg[s:t], self.exp_avg_sq[s:t], coef, lr, b1, b2, self.eps,
                            self.weight_decay if decay else 0.0, self.step_count,
                            sr_seed=(0x5EED + 7919 * self.step_count) & 0x7FFFFFFF if self.stochastic_rounding else 0,
                            sr_offset=s)

        if getattr(self, "overlap", False):
            st = self._stream
            st.wait_stream(torch.cuda.current_stream())
            coef.record_stream(st)
            self._coef = coef
            with torch.cuda.stream(st):
                for rs, ev in zip(self._groups, self._events):
                    for s, t, decay in rs:
                        upd(s, t, decay)
                    ev.record(st)
            self._pending = True
            return norm
        for s, t, decay in e.regions:
            upd(s, t, decay)
        return norm

    def state_dict(self) -> Dict:
        self.synchronize()
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "master": self.master, "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd: Dict):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])  # copy_ converts between fp32 / bf16 state checkpoints
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        if self.master is not None:
            if sd.get("master") is not None:
                self.master.copy_(sd["master"])
            else:
                self.master.copy_(self.engine.param_flat.float())


def get_schedule(name: str, num_training_steps: int, num_warmup_steps: int = 0, **kw) -> Callable[[int], float]:
    """LR multiplier as a function of the optimizer step (HF transformers semantics)."""
    name = (name or "linear").lower()
    W, T = max(0, num_warmup_steps), max(1, num_training_steps)

    def warm(s):
        return s / max(1, W)

    if name == "linear":
        return lambda s: warm(s) if s < W else max(0.0, (T - s) / max(1, T - W))
    if name == "cosine":
        cycles = kw.get("num_cycles", 0.5)

        def f(s):
            if s < W:
                return warm(s)
            p = (s - W) / max(1, T - W)
            return max(0.0, 0.5 * (1.0 + math.cos(math.pi * cycles * 2.0 * p)))
        return f
    if name == "cosine_with_min_lr":
        min_ratio = kw.get("min_lr_rate", 0.1)

        def g(s):
            if s < W:
                return warm(s)
            p = min(1.0, (s - W) / max(1, T - W))
            return min_ratio + (1 - min_ratio) * 0.5 * (1.0 + math.cos(math.pi * p))
        return g
    if name == "constant":
        return lambda s: 1.0
    if name == "constant_with_warmup":
        return lambda s: warm(s) if s < W else 1.0
    raise ValueError(f"unknown lr_scheduler_type {name!r}")


class LRScheduler:
    def __init__(self, optimizer: FlatAdamW, fn: Callable[[int], float]):
        self.optimizer = optimizer
        self.fn = fn
        self.base_lr = optimizer.lr
        self.last_step = 0

    def get_lr(self, step: Optional[int] = None) -> float:
        return self.base_lr * self.fn(self.last_step if step is None else step)

    def step(self):
        self.last_step += 1

    def state_dict(self):
        return {"last_step": self.last_step, "base_lr": self.base_lr}

    def load_state_dict(self, sd):
        self.last_step = int(sd["last_step"])
        self.base_lr = float(sd.get("base_lr", self.base_lr))
