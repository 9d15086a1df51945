"""Flat AdamW + LR schedules (reference T3/T4/T5).

The reference runs HF's default ``adamw_torch(_fused)`` over bf16 parameters with
``lr = LEARNING_RATE * WORLD_SIZE`` (training.py:263), betas (0.9, 0.999), eps 1e-8, wd 0, and
``lr_scheduler_type="linear"`` (decay to 0, no warmup). Here the update is ONE fused HIP kernel
per weight-decay region over the DDP engine's flat buffers. Trainer default (SFTConfig): the reference's
state — bf16 parameters updated in place and Adam moments in the parameter dtype (bf16), every bf16
write-back stochastically rounded; fp32 moments and an fp32 master copy are options. Gradient clipping
(max_grad_norm) is a sum of squares produced during backward (or a flat pass); the clip coefficient never
leaves the GPU.
"""
from __future__ import annotations

import contextlib
import math
from typing import Callable, Dict, Optional

import torch

from .. import ops


def _update_stream(device: torch.device):
    """Side stream of the overlapped optimizer update (restricting it to a few CUs with a CU-masked stream measured
    neutral to negative, profiles/r2_gemm_pingpong.md)."""
    return torch.cuda.Stream(device=device)


def _state_dtype(state_dtype, engine, master_weights: bool = False) -> torch.dtype:
    """Adam moment dtype: "auto" = the parameter dtype (torch AdamW's state follows its parameters: bf16 for the
    reference's bf16 model, training.py:99) — except with an fp32 master copy, where the update runs without
    stochastic rounding and a round-to-nearest bf16 exp_avg_sq would stall (beta2 = 0.999 moves it by less than
    half a bf16 ulp per step), so "auto" means fp32 there; "bf16" / "fp32", or a torch dtype."""
    if isinstance(state_dtype, str):
        if state_dtype == "auto":
            if master_weights:
                return torch.float32
            return engine.dtype if engine.dtype in (torch.float32, torch.bfloat16) else torch.float32
        state_dtype = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
                       "bfloat16": torch.bfloat16}[state_dtype]
    return state_dtype


class _StreamPoint:
    """Work-like handle for an update with no collective behind it: ``wait()`` makes the current
    stream wait for the side stream up to the point where the handle was created."""

    def __init__(self, stream):
        self._ev = torch.cuda.Event()
        self._ev.record(stream)

    def wait(self):
        torch.cuda.current_stream().wait_event(self._ev)


class FlatAdamW:
    def __init__(self, engine, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 master_weights: bool = True, stochastic_rounding: bool = True, state_dtype="auto"):
        """``state_dtype`` = dtype of exp_avg / exp_avg_sq: "auto" (the parameter dtype, like torch), fp32 or bf16 —
        what torch's AdamW keeps for the reference's bf16 parameters (training.py:99) — stored with stochastic
        rounding (unbiased) when ``stochastic_rounding`` is on; 8 fewer HBM bytes per parameter than fp32."""
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
        state_dtype = _state_dtype(state_dtype, engine, master_weights)
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
        self._stream = _update_stream(e.device)
        self._pending = False
        self._hooks = []

        # layer i's forward waits for the update of its own parameters (group i + 1; group 0 = the embedding) — one
        # stream-wait packet per layer; the in-order update stream normally runs layers ahead of the forward
        nl = len(inner.layers)

        def waiter(i):
            def hook(*_a, **_k):
                if self._pending:
                    torch.cuda.current_stream().wait_event(self._events[i])
            return hook

        self._hooks.append(model.register_forward_pre_hook(waiter(0)))
        for i, layer in enumerate(inner.layers):
            self._hooks.append(layer.register_forward_pre_hook(waiter(min(i + 1, nl))))
        self._hooks.append(inner.layers[-1].register_forward_hook(waiter(len(groups) - 1)))
        ops.register_param_sync(self.synchronize)  # reads of many layers' parameters at once (LoRA wide refresh)
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
        norm2 = e.grad_norm_sq()  # computed bucket by bucket during backward (replicated buckets)
        if norm2 is not None:
            norm = norm2.sqrt()
            coef = ((max_grad_norm / (norm + 1e-6)).clamp(max=1.0) if max_grad_norm and max_grad_norm > 0
                    else torch.ones_like(norm))
        else:
            norm, coef = ops.grad_norm_flat([e.grad_flat], max_grad_norm if max_grad_norm else 0.0)
        self.last_grad_norm = norm
        b1, b2 = self.betas
        # the parameters change in place through a raw-pointer kernel: tell caches of parameter copies (LoRA's wide
        # weight, ops.fused._sync_wide) that they are stale
        ops.bump_param_epoch()

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

    # ------------------------------------------------------------------ checkpoints (per parameter)
    def _full_state(self, key: str, dst: Optional[int] = None) -> Optional[torch.Tensor]:
        """The whole-model flat tensor of ``key`` in this engine's layout (collective under ZeRO-1; built only on
        rank ``dst`` when given)."""
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "master": self.master}[key]

    def _state_ranges(self):
        """(global_start, global_end, local_offset) of the flat state this rank holds."""
        return [(0, self.engine.numel, 0)]

    def _collective_state(self) -> bool:
        return False  # replicated state: every rank already holds all of it

    def state_dict(self, dst: Optional[int] = 0) -> Dict:
        """Adam state keyed by PARAMETER NAME (``param_state[name] = {exp_avg, exp_avg_sq, master}`` with the
        parameter's shape), so a checkpoint resumes at any world size / bucket plan: the flat layout pads
        buckets to multiples of world_size pages and is therefore world-size dependent. Tensors are host copies.

        ``dst`` (default 0): only that rank builds the state; every other rank returns ``{}`` without allocating a
        full host (or device) copy — under ZeRO-1 they still join the collectives that bring their shards to
        ``dst`` (every rank must call), replicated state needs no communication at all. ``dst=None``: every rank
        builds the full state (the round-2 behaviour)."""
        self.synchronize()
        e = self.engine
        self.last_state_dict_host_bytes = 0
        mine = dst is None or e.rank == dst
        if not mine and not self._collective_state():
            return {}
        full = {}
        for k in ("exp_avg", "exp_avg_sq", "master"):
            t = self._full_state(k, dst)
            if not mine:
                continue
            full[k] = None if t is None else t.detach().cpu()
            if t is not None:
                self.last_state_dict_host_bytes += t.numel() * t.element_size()
        if not mine:
            return {}
        ps = {}
        for p, o, n, _ in e.layout:
            ps[e.param_names[id(p)]] = {k: (None if v is None else v[o:o + n].view(p.shape)) for k, v in full.items()}
        return {"format": "sftamd-adamw-v2", "step": self.step_count, "param_state": ps,
                "state_dtype": str(self.state_dtype).replace("torch.", ""), "lr": self.lr, "betas": self.betas,
                "eps": self.eps, "weight_decay": self.weight_decay, "saved_world_size": e.world_size}

    def load_state_dict(self, sd: Dict):
        e = self.engine
        self.step_count = int(sd["step"])
        ranges = self._state_ranges()
        dsts = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "master": self.master}
        if "param_state" not in sd:  # round-1 flat format: only valid for the same layout
            if sd["exp_avg"].numel() != e.numel:
                raise ValueError(f"flat optimizer state of {sd['exp_avg'].numel()} elements does not match this "
                                 f"layout ({e.numel}); re-save with the per-parameter format")
            for s, t, lo in ranges:
                for k in ("exp_avg", "exp_avg_sq"):
                    dsts[k][lo:lo + t - s].copy_(sd[k][s:t])
                if self.master is not None:
                    src = sd.get("master")
                    self.master[lo:lo + t - s].copy_(src[s:t] if src is not None else e.param_flat[s:t].float())
            return
        ps = sd["param_state"]
        missing = [e.param_names[id(p)] for p, _, _, _ in e.layout if e.param_names[id(p)] not in ps]
        if missing:
            raise KeyError(f"optimizer checkpoint has no state for {missing[:4]}{'...' if len(missing) > 4 else ''}")
        for p, o, n, _ in e.layout:
            st = ps[e.param_names[id(p)]]
            for s, t, lo in ranges:
                a, b = max(s, o), min(t, o + n)
                if a >= b:
                    continue
                for k in ("exp_avg", "exp_avg_sq", "master"):
                    dst = dsts[k]
                    if dst is None:
                        continue
                    src = st.get(k)
                    if src is None:  # no saved master: start it from the current (bf16) parameters
                        src = e.param_flat[o:o + n].float()
                    dst[lo + a - s:lo + b - s].copy_(src.reshape(-1)[a - o:b - o].to(dst.device, dst.dtype))


class ShardedAdamW(FlatAdamW):
    """ZeRO-1 AdamW over the DDP engine's flat buffers (engine built with ``shard=True``).

    Each rank owns 1/world_size of every gradient bucket: the engine reduce-scatters a bucket the moment
    it completes in backward (half the bytes of the all-reduce on the backward critical path), this
    optimizer updates only the owned slices — moments and master copy exist for those slices only, so
    optimizer HBM traffic and memory shrink by world_size — and the updated parameter slices are
    all-gathered back, bucket by bucket in FORWARD order (embedding first), on the collective stream
    while the next forward runs: a layer's forward pre-hook waits only for its own buckets.
    The update itself is the same fused HIP kernel, with the stochastic-rounding stream keyed by the
    GLOBAL element index, so a sharded run rounds exactly like the replicated one.
    Checkpoints hold the full (gathered) per-parameter state, interchangeable with ``FlatAdamW``'s and
    loadable at any world size."""

    def __init__(self, engine, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 master_weights: bool = True, stochastic_rounding: bool = True, state_dtype="auto"):
        if not engine.shard:
            raise ValueError("ShardedAdamW needs a DDPEngine built with shard=True")
        self.engine = engine
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.master_weights = master_weights
        self.stochastic_rounding = stochastic_rounding and not master_weights
        self.step_count = 0
        self.state_dtype = state_dtype = _state_dtype(state_dtype, engine, master_weights)
        e = engine
        # owned slice of every bucket -> offset in the local (sharded) state buffers
        self.slices = []  # (bucket, start, end, local_offset, decay)
        off = 0
        for b in e.buckets:
            s, t = e.shard_range(b)
            decay = next(d for rs, rt, d in e.regions if rs <= b.start < rt)
            self.slices.append((b, s, t, off, decay))
            off += t - s
        self.local_numel = off
        dev = e.device
        self.exp_avg = torch.zeros(off, dtype=state_dtype, device=dev)
        self.exp_avg_sq = torch.zeros(off, dtype=state_dtype, device=dev)
        self.master = None
        if master_weights:
            self.master = torch.empty(off, dtype=torch.float32, device=dev)
            for _, s, t, lo, _ in self.slices:
                self.master[lo:lo + t - s].copy_(e.param_flat[s:t].float())
        self.last_grad_norm = None
        self.overlap = False
        self._ag = {}
        self._pending = False

    # ------------------------------------------------------------------ gather under the next forward
    def enable_overlap(self, model) -> bool:
        """Forward pre-hooks wait for the all-gathers of the buckets holding each module's parameters."""
        e = self.engine
        inner = model.model

        def buckets_of(params):
            out = []
            for p in params:
                for b in e.param_bucket.get(id(p), ()):
                    if b.index not in out:
                        out.append(b.index)
            return out

        groups = [buckets_of([inner.embed_tokens])]
        for layer in inner.layers:
            groups.append(buckets_of(list(layer.parameters())))
        head = list(inner.norm.parameters()) + ([model.lm_head] if model.lm_head is not None else [])
        groups.append(buckets_of(head))
        self._wait_groups = groups

        last = len(groups) - 1

        def waiter(i):
            def hook(*_a, **_k):
                if self._pending:
                    for bi in self._wait_groups[i]:
                        w = self._ag.pop(bi, None)
                        if w is not None:
                            w.wait()
                    if i == last:  # buckets outside every group: done before the next backward writes grads
                        self.synchronize()
            return hook

        self._hooks = [model.register_forward_pre_hook(waiter(0))]
        for i, layer in enumerate(inner.layers):
            self._hooks.append(layer.register_forward_pre_hook(waiter(i + 1)))
        self._hooks.append(inner.layers[-1].register_forward_hook(waiter(last)))
        self._stream = _update_stream(e.device) if e.device.type == "cuda" else None
        ops.register_param_sync(self.synchronize)
        self.overlap = True
        return True

    def synchronize(self):
        if self._ag:
            for w in self._ag.values():
                if w is not None:
                    w.wait()
            self._ag = {}
        self._pending = False

    @torch.no_grad()
    def step(self, lr: Optional[float] = None, max_grad_norm: Optional[float] = None):
        lr = self.lr if lr is None else lr
        self.step_count += 1
        e = self.engine
        self.synchronize()
        # global grad norm: sum of squares of the owned (reduced) slices, all-reduced (one float)
        norm2 = e.grad_norm_sq()  # owned slices, summed bucket by bucket during backward
        if norm2 is None:
            # replicated buckets (sparse tied embedding) are whole on every rank: counted once, on rank 0
            owned = [e.grad_flat[s:t] for b, s, t, _, _ in self.slices if t > s and (not b.replicated or e.rank == 0)]
            norm2 = ops.sumsq_list(owned).reshape(1) if owned else torch.zeros(1, device=e.device)
        if e.world_size > 1:
            e.all_reduce_small_(norm2)
        norm = norm2.sqrt()
        coef = (max_grad_norm / (norm + 1e-6)).clamp(max=1.0) if max_grad_norm else torch.ones_like(norm)
        self.last_grad_norm = norm
        b1, b2 = self.betas
        ops.bump_param_epoch()  # see FlatAdamW.step
        seed = (0x5EED + 7919 * self.step_count) & 0x7FFFFFFF if self.stochastic_rounding else 0
        # Overlapped: updates AND gathers are issued from a side stream, so the next forward only waits
        # for the buckets each layer reads (update -> gather chain per bucket), not for the whole update.
        st = self._stream if (self.overlap and getattr(self, "_stream", None) is not None) else None
        ctx = contextlib.nullcontext()
        if st is not None:
            st.wait_stream(torch.cuda.current_stream(e.device))
            coef.record_stream(st)
            ctx = torch.cuda.stream(st)
        with ctx:
            # forward order (the embedding's bucket is the LAST one in backward-ready layout): each bucket's
            # gather is issued right after its update, so the first layers' parameters come back first; replicated
            # buckets (the sparse-mode tied embedding: first in the layout, needed by the first forward op, no
            # gather) are updated before everything else
            order = [x for x in self.slices if x[0].replicated] + [x for x in reversed(self.slices)
                                                                  if not x[0].replicated]
            for b, s, t, lo, decay in order:
                n = t - s
                if n:
                    ops.adamw_flat_(e.param_flat[s:t], e.grad_flat[s:t],
                                    None if self.master is None else self.master[lo:lo + n],
                                    self.exp_avg[lo:lo + n], self.exp_avg_sq[lo:lo + n], coef, lr, b1, b2, self.eps,
                                    self.weight_decay if decay else 0.0, self.step_count, sr_seed=seed, sr_offset=s)
                w = e.gather_params(b, async_op=True)
                if w is None and st is not None:
                    w = _StreamPoint(st)
                if w is not None:
                    self._ag[b.index] = w
        self._pending = bool(self._ag)
        if not self.overlap:
            self.synchronize()
        return norm

    # ------------------------------------------------------------------ checkpoints: full (gathered) state
    def _collective_state(self) -> bool:
        return self.engine.world_size > 1

    def _full_state(self, key: str, dst: Optional[int] = None) -> Optional[torch.Tensor]:
        """The full flat state ``key``: all-gathered onto every rank (``dst=None``) or GATHERED onto rank ``dst``
        only — the other ranks send their owned slice of each bucket and never allocate the full tensor (a 3B model's
        bf16 moments are ~6 GB per tensor: at N = 8 a full copy on every rank would be ~48 GB per state tensor)."""
        import torch.distributed as dist
        local = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "master": self.master}[key]
        if local is None:
            return None
        e = self.engine
        if dst is None or e.world_size == 1:
            full = torch.zeros(e.numel, dtype=local.dtype, device=e.device)
            for b, s, t, lo, _ in self.slices:
                full[s:t].copy_(local[lo:lo + t - s])
                if e.world_size > 1 and not b.replicated:
                    dist.all_gather_into_tensor(full[b.start:b.end], full[s:t], group=e.pg)
            return full
        me = e.rank == dst
        full = torch.zeros(e.numel, dtype=local.dtype, device=e.device) if me else None
        for b, s, t, lo, _ in self.slices:
            if b.replicated:  # whole on every rank: the destination has it already
                if me:
                    full[s:t].copy_(local[lo:lo + t - s])
                continue
            n = t - s
            parts = [full[b.start + r * n:b.start + (r + 1) * n] for r in range(e.world_size)] if me else None
            dist.gather(local[lo:lo + n].contiguous(), parts, dst=dst, group=e.pg)
        return full

    def _state_ranges(self):
        return [(s, t, lo) for _, s, t, lo, _ in self.slices]


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
