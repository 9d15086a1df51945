"""Native DDP engine: flat bucketed gradients, all-reduce overlapped with backward.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as configured by the reference
(``find_unused_parameters=False, bucket_cap_mb=50``, ``training.py:249-256``) with a design
that maps to MI355X + RCCL over xGMI:

* every trainable parameter (and its gradient) lives in ONE flat buffer, laid out in the order
  gradients become ready in backward (reverse registration order); parameters become views.
  The gradient buffer is bucketed in place (bucket == contiguous slice), so there is no
  copy-into-bucket / copy-back (the c10d Reducer's K13 traffic) and the optimizer is a single
  flat kernel;
* weight gradients are accumulated directly into ``param.main_grad`` (views of the flat
  gradient buffer) by the fused ops; a parameter's ready-hook fires when all of its forward
  uses have been back-propagated (tied embedding: lm_head GEMM + embedding backward);
* on the synchronising micro-batch, a bucket is all-reduced (RCCL SUM, async, on the process
  group's stream, event-ordered after the producing kernels) as soon as it is complete;
  buckets launch strictly in index order, so every rank issues the same collective sequence;
* gradient accumulation = ``no_sync`` on all but the last micro-batch: no communication at all
  (one all-reduce round per optimizer step, the reference's GA semantics, lib trainer.py:1749);
* all ranks build identical weights from the same seed / checkpoint, so the 6 GB rank-0
  broadcast of the reference's DDP constructor (C3) is skipped unless asked for;
* ``shard=True`` (ZeRO-1, train/optim.py ``ShardedAdamW``): a completed bucket is REDUCE-SCATTERED
  in place (each rank receives the summed slice it owns — half the bytes of an all-reduce on the
  backward critical path), each rank updates only its slice, and the updated parameter slices are
  ALL-GATHERED back bucket by bucket under the next forward. The bucket padding below makes every
  slice an equal, 128-byte-aligned 1/world_size of its bucket.

Bucket sizing for xGMI (``plan_bucket_mb``): each MI355X has 7 point-to-point xGMI links, one per
peer, and RCCL stripes a collective over channels that use all N-1 of them, so a reduce-scatter of S
bytes costs about ``alpha + S / (N * L)`` (``alpha`` = per-call latency, ``L`` = effective per-link
bandwidth). The cap is the smallest S whose latency share is <= ~15% (``S >= 5.7 * alpha * N * L``),
clamped to [16, 256] MB and to >= 8 buckets over the model, then rounded so every one of the N shards is a
whole number of 4 KiB pages. ``alpha`` and ``L`` are MEASURED at startup (``measure_link``: reduce-scatters of
two sizes, the max over ranks, ``fit_link``; the trainer does this when no cap is given) and fall back to the
modelled 30 us / 100 GB/s (env ``SFTAMD_XGMI_ALPHA_US`` / ``SFTAMD_XGMI_LINK_GBPS``): 33 / 65 / 130 MB at
N = 2 / 4 / 8 — grown with N because each rank moves only 1/N of a bucket per link (the reference's 50 MB cap,
``training.py:253``, was sized for a single TCP ring). The first bucket stays small (4 MB) so
communication starts early in backward.

Oversized parameters (larger than twice the cap, e.g. Llama-3-8B's 1 GB untied lm_head or the 525 MB
tied SmolLM3 embedding) are SPLIT across consecutive buckets at shard-aligned cut points: every bucket
that holds a slice of the parameter counts it, and the parameter's ready signal completes all of them,
so no collective is larger than ~2 caps and ZeRO-1 state / gathers stay evenly spread.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist


@dataclass
class Bucket:
    index: int
    start: int
    end: int
    params: List[torch.nn.Parameter] = field(default_factory=list)
    ready: bool = False
    launched: bool = False
    work: Optional[object] = None
    replicated: bool = False  # tied-embedding buckets in sparse mode: all-reduced and updated on every rank


def _plan_python(sizes, region, tied, align, pad_unit, cap, first_cap, split_at):
    """Pure-Python twin of csrc/ddp_reducer.cpp ddp_plan (same packed result): used when the extension is not
    built, and by the tests that pin the native planner to it."""
    def rup(x, m):
        return (x + m - 1) // m * m

    np_ = len(sizes)
    offset = [0] * np_
    own = [[] for _ in range(np_)]
    bstart, bend, brepl, regions = [], [], [], []
    off = n_split = 0
    i = 0
    while i < np_:
        reg = region[i]
        j = i
        while j < np_ and region[j] == reg:
            j += 1
        off = rup(off, pad_unit)
        rs = off

        def open_(at):
            bstart.append(at)
            bend.append(at)
            brepl.append(0)
            return len(bstart) - 1
        cur, cur_params = open_(off), 0
        for k in range(i, j):
            sz = rup(sizes[k], align)
            limit = first_cap if cur == 0 else cap
            if cur_params and off + sz - bstart[cur] > limit:
                off = rup(off, pad_unit)
                bend[cur] = off
                cur, cur_params = open_(off), 0
            offset[k] = off
            own[k].append(cur)
            cur_params += 1
            end = off + sz
            if split_at > 0 and sz > split_at:
                n_split += 1
                while end - bstart[cur] > split_at:
                    cut = (bstart[cur] + cap) // pad_unit * pad_unit
                    bend[cur] = cut
                    cur, cur_params = open_(cut), 1
                    own[k].append(cur)
            off = end
            if k == tied:
                for b in own[k]:
                    brepl[b] = 1
                off = rup(off, pad_unit)
                bend[cur] = off
                cur, cur_params = open_(off), 0
        off = rup(off, pad_unit)
        bend[cur] = off
        if cur_params == 0:
            bstart.pop(), bend.pop(), brepl.pop()
        regions += [rs, off, 1 if reg == 0 else 0]
        i = j
    owner_ptr = [0]
    for o in own:
        owner_ptr.append(owner_ptr[-1] + len(o))
    return ([off, len(bstart), np_, len(regions) // 3] + offset + bstart + bend + brepl + owner_ptr
            + [b for o in own for b in o] + regions + [n_split])


def _native():
    from ..ops import _ext
    return _ext.ops() if _ext.load() else None


def ddp_plan(sizes, region, tied, align, pad_unit, cap, first_cap, split_at) -> List[int]:
    """Bucket plan of the flat gradient buffer (csrc/ddp_reducer.cpp; Python twin when the extension is absent)."""
    ops = _native()
    if ops is not None:
        return list(ops.ddp_plan(sizes, region, tied, align, pad_unit, cap, first_cap, split_at))
    return _plan_python(sizes, region, tied, align, pad_unit, cap, first_cap, split_at)


class ReadyTracker:
    """Per-bucket pending counts and in-order launch (csrc/ddp_reducer.cpp ddp_tracker_*; the c10d Reducer's
    bookkeeping), with a Python twin when the extension is absent (``native=False`` forces it)."""

    def __init__(self, owner_ptr, owners, n_buckets: int, native: Optional[bool] = None):
        self._ops = _native() if native is not False else None
        if native and self._ops is None:
            raise RuntimeError("native DDP tracker requested but the extension is not loaded")
        self.n = n_buckets
        if self._ops is not None:
            self._id = self._ops.ddp_tracker_create(list(owner_ptr), list(owners), n_buckets)
        else:
            self._ptr, self._own = list(owner_ptr), list(owners)
            self._init = [0] * n_buckets
            for b in self._own:
                self._init[b] += 1
            self.reset()

    @property
    def native(self) -> bool:
        return self._ops is not None

    def reset(self):
        if self._ops is not None:
            self._ops.ddp_tracker_reset(self._id)
            return
        self._pending = list(self._init)
        self._marked = [False] * (len(self._ptr) - 1)
        self._ready = [False] * self.n
        self._next = 0

    def mark(self, param: int) -> List[int]:
        if self._ops is not None:
            return list(self._ops.ddp_tracker_mark(self._id, param))
        if self._marked[param]:
            raise RuntimeError(f"DDP parameter {param} signalled ready twice in one backward")
        self._marked[param] = True
        for b in self._own[self._ptr[param]:self._ptr[param + 1]]:
            if self._pending[b] <= 0:
                raise RuntimeError(f"DDP bucket {b}: more ready signals than parameters")
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
        out = []
        while self._next < self.n and self._ready[self._next]:
            out.append(self._next)
            self._next += 1
        return out

    def drain(self) -> List[int]:
        if self._ops is not None:
            return list(self._ops.ddp_tracker_drain(self._id))
        rest = list(range(self._next, self.n))
        self._next = self.n
        return rest

    def pending(self) -> List[int]:
        if self._ops is not None:
            return list(self._ops.ddp_tracker_pending(self._id))
        return list(self._pending)

    def __del__(self):
        ops = getattr(self, "_ops", None)
        if ops is not None:
            try:
                ops.ddp_tracker_destroy(self._id)
            except Exception:
                pass


def _no_decay(name: str, p: torch.Tensor) -> bool:
    return p.dim() < 2 or "norm" in name or name.endswith(".bias")


SHARD_PAGE_BYTES = 4096  # every reduce-scatter / all-gather shard is a whole number of 4 KiB pages


def plan_bucket_mb(world_size: int, total_bytes: int = 0, alpha_us: Optional[float] = None,
                   link_gbps: Optional[float] = None) -> float:
    """Gradient-bucket cap (MB) for a reduce-scatter / all-reduce over N ranks on the xGMI full mesh
    (see the module docstring): latency share <= ~15%, clamped to [16, 256] MB and to >= 8 buckets."""
    import os
    alpha = (alpha_us if alpha_us is not None else float(os.environ.get("SFTAMD_XGMI_ALPHA_US", "30"))) * 1e-6
    link = (link_gbps if link_gbps is not None else float(os.environ.get("SFTAMD_XGMI_LINK_GBPS", "100"))) * 1e9
    n = max(1, world_size)
    mb = 5.7 * alpha * n * link / 2 ** 20
    if total_bytes > 0:
        mb = min(mb, max(16.0, total_bytes / 8 / 2 ** 20))
    return float(min(256.0, max(16.0, mb)))


def fit_link(points, world_size: int, strict: bool = False):
    """(alpha_us, link_gbps) of ``t = alpha + S / (N L)`` through measured (bytes, seconds) reduce-scatter points
    (least squares over >= 2 sizes; the slope is 1 / (N L): each rank moves 1/N of the buffer per link). Guarded
    against noise: alpha >= 1 us, L in [1, 1000] GB/s. ``strict``: None instead of a fit above 1000 GB/s (a flat or
    negative slope from a noisy probe would otherwise pin L at 1000 GB/s and the bucket cap at its ceiling — the
    caller then keeps the modelled plan)."""
    pts = sorted((float(b), float(t)) for b, t in points)
    if len(pts) < 2 or pts[-1][0] <= pts[0][0]:
        raise ValueError("fit_link needs >= 2 distinct message sizes")
    n = len(pts)
    mx = sum(b for b, _ in pts) / n
    my = sum(t for _, t in pts) / n
    sxx = sum((b - mx) ** 2 for b, _ in pts)
    slope = sum((b - mx) * (t - my) for b, t in pts) / sxx
    slope = max(slope, 1e-15)
    alpha = max(1e-6, my - slope * mx)
    link = 1.0 / (slope * max(1, world_size)) / 1e9
    if strict and link > 1000.0:  # the clamp that matters: it would set the bucket cap to its ceiling
        return None
    return alpha * 1e6, float(min(1000.0, max(1.0, link)))


def measure_link(world_size: int, device, group=None, sizes_mb=(4.0, 32.0), iters: int = 7):
    """Startup probe of the gradient collective: in-place reduce-scatter of bf16 buffers of ``sizes_mb``, each call
    timed on every rank (two warm-up calls first); the MAX over ranks of each size's MEDIAN time (robust to one slow
    call; every rank fits the SAME alpha / L and builds the same bucket plan). Returns [(bytes, seconds), ...]."""
    if world_size <= 1:
        return []
    import time
    on_gpu = torch.device(device).type == "cuda"
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    rank = dist.get_rank(group)
    out = []
    for mb in sizes_mb:
        n = max(world_size * 64, int(mb * 2 ** 20 / 2) // (world_size * 64) * (world_size * 64))
        buf = torch.ones(n, dtype=torch.bfloat16, device=device)
        part = buf[rank * (n // world_size):(rank + 1) * (n // world_size)]
        for _ in range(2):  # warm (RCCL channel setup on the first call)
            dist.reduce_scatter_tensor(part, buf, group=group)
        sync()
        dist.barrier(group=group)
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            dist.reduce_scatter_tensor(part, buf, group=group)
            sync()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out.append([n * 2, ts[len(ts) // 2]])
        del buf, part
    t = torch.tensor([p[1] for p in out], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [(p[0], float(v)) for p, v in zip(out, t.tolist())]


class DDPEngine:
    def __init__(self, model: torch.nn.Module, world_size: int = 1, rank: int = 0,
                 bucket_cap_mb: Optional[float] = None, first_bucket_mb: float = 4.0,
                 grad_dtype: Optional[torch.dtype] = None,
                 broadcast_params: bool = False, align: int = 64, process_group=None,
                 no_decay_fn: Callable[[str, torch.Tensor], bool] = _no_decay, shard: bool = False,
                 track_norm: Optional[bool] = None, split_oversized: bool = True, tied_sparse: Optional[bool] = None,
                 link: Optional[tuple] = None):
        """``link``: (alpha_us, link_gbps) of the collective as measured at startup (``fit_link(measure_link(...))``);
        with no ``bucket_cap_mb`` the bucket cap is planned from it instead of the modelled defaults."""
        self.model = model
        self.world_size = world_size
        self.rank = rank
        self.pg = process_group
        self.shard = shard
        self.sync_grads = True
        named = []
        seen = set()
        for n, p in model.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                named.append((n, p))
        if not named:
            raise ValueError("no trainable parameters")
        # backward-ready order = reverse registration; decay params first, no-decay after
        rev = list(reversed(named))
        if track_norm is None:
            track_norm = os.environ.get("SFTAMD_NORM_IN_BWD", "0") == "1"
        # Sparse tied-embedding gradient (world > 1, tied lm_head / embedding): the tied weight's gradient has a
        # dense part (lm_head wgrad, the FIRST weight gradient of backward) and a sparse part (embedding backward,
        # the LAST op of backward, only the rows of the step's tokens). Dense mode ships the sum as the last
        # buckets, exposed after backward (and, under ZeRO-1, gathered again before the next forward's first op).
        # Sparse mode: the tied weight leads the layout in buckets of its own, all-reduced as soon as the lm_head
        # wgrad lands (overlapped with the whole backward); the embedding backward hands (unique ids, summed rows)
        # to the engine instead, all ranks all-gather those (N x <= tokens x hidden) after backward and add them in
        # rank order; the tied weight is then updated on every rank (replicated, no ZeRO all-gather).
        tied_w = None
        inner = getattr(model, "model", None)
        if getattr(model, "lm_head", 0) is None and inner is not None and hasattr(inner, "embed_tokens"):
            tied_w = inner.embed_tokens if inner.embed_tokens.requires_grad else None
        if tied_sparse is None:
            tied_sparse = os.environ.get("SFTAMD_TIED_SPARSE", "1") == "1"
        self.tied_sparse = bool(tied_sparse and tied_w is not None and world_size > 1 and not track_norm)
        self.tied_param = tied_w if self.tied_sparse else None
        if self.tied_sparse:
            rev = [(n, p) for n, p in rev if p is tied_w] + [(n, p) for n, p in rev if p is not tied_w]
        decay = [(n, p) for n, p in rev if not no_decay_fn(n, p)]
        nodecay = [(n, p) for n, p in rev if no_decay_fn(n, p)]
        self.param_names: Dict[int, str] = {id(p): n for n, p in named}
        dtype = named[0][1].dtype
        dev = named[0][1].device
        self.dtype = dtype
        self.device = dev
        self.grad_dtype = grad_dtype or dtype
        esz = torch.empty((), dtype=self.grad_dtype).element_size()
        # bucket boundaries: multiples of world_size * (4 KiB of elements) -> equal, page-aligned shards
        pad_unit = max(align, SHARD_PAGE_BYTES // esz) * max(1, world_size)
        self.plan_source = "user" if bucket_cap_mb else ("probe" if link else "model")
        self.link_alpha_us = float(link[0]) if link else float(os.environ.get("SFTAMD_XGMI_ALPHA_US", "30"))
        self.link_gbps = float(link[1]) if link else float(os.environ.get("SFTAMD_XGMI_LINK_GBPS", "100"))
        if not bucket_cap_mb:
            bucket_cap_mb = plan_bucket_mb(world_size, sum(p.numel() for _, p in named) * esz,
                                           alpha_us=self.link_alpha_us, link_gbps=self.link_gbps)
        self.bucket_cap_mb = float(bucket_cap_mb)
        cap = max(pad_unit, int(bucket_cap_mb * 1024 * 1024 / esz))
        first_cap = max(pad_unit, int(first_bucket_mb * 1024 * 1024 / esz))
        split_at = 2 * cap if split_oversized else None
        ordered = decay + nodecay
        tied_idx = next((i for i, (_, p) in enumerate(ordered) if p is self.tied_param), -1)
        plan = ddp_plan([p.numel() for _, p in ordered], [0] * len(decay) + [1] * len(nodecay), tied_idx, align,
                        pad_unit, cap, first_cap, split_at or 0)
        numel, nb, np_, nr = plan[:4]
        k = 4
        offsets = plan[k:k + np_]
        k += np_
        bstart, bend, brepl = plan[k:k + nb], plan[k + nb:k + 2 * nb], plan[k + 2 * nb:k + 3 * nb]
        k += 3 * nb
        owner_ptr = plan[k:k + np_ + 1]
        k += np_ + 1
        owners = plan[k:k + owner_ptr[-1]]
        k += owner_ptr[-1]
        regs = plan[k:k + 3 * nr]
        self.num_split_params = plan[k + 3 * nr]
        self.buckets: List[Bucket] = [Bucket(index=i, start=bstart[i], end=bend[i], replicated=bool(brepl[i]))
                                      for i in range(nb)]
        self.layout: List[tuple] = []  # (param, offset, numel, region)
        self.param_bucket: Dict[int, List[Bucket]] = {}
        self._param_index: Dict[int, int] = {}
        for i, (_, p) in enumerate(ordered):
            self.layout.append((p, offsets[i], p.numel(), "decay" if i < len(decay) else "no_decay"))
            own = [self.buckets[b] for b in owners[owner_ptr[i]:owner_ptr[i + 1]]]
            for b in own:
                b.params.append(p)
            self.param_bucket[id(p)] = own
            self._param_index[id(p)] = i
        self.regions = [(regs[3 * r], regs[3 * r + 1], bool(regs[3 * r + 2])) for r in range(nr)]
        self._tracker = ReadyTracker(owner_ptr, owners, nb)
        self.numel = numel
        self.param_flat = torch.zeros(self.numel, dtype=dtype, device=dev)
        self.grad_flat = torch.zeros(self.numel, dtype=self.grad_dtype, device=dev)
        with torch.no_grad():
            for p, o, n, _ in self.layout:
                self.param_flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.param_flat[o:o + n].view(p.shape)
                p.main_grad = self.grad_flat[o:o + n].view(p.shape)
                p.grad = None
        self._comm_events = []
        self.last_launched = -1  # index of the last bucket whose collective was issued (heartbeat / hang triage)
        # gradient-norm partials computed during backward (SFTAMD_NORM_IN_BWD=1): one sum of squares per
        # bucket (its reduced / owned slice), on a side stream as soon as the bucket is complete, instead of
        # a serial pass over every gradient after backward. Measured on MI355X (bench.py, interleaved): 96.0
        # vs 96.2-96.3 samples/s without — the concurrent HBM pass slows the backward GEMMs as much as it
        # saves, so it is off by default.
        self.track_norm = bool(track_norm)
        self._sparse = None
        self.sparse_exchanges = 0  # synchronising passes whose tied-embedding rows went through the sparse path
        self.sparse_cap = 0  # host-known upper bound of one pass's token count (trainer); 0 = measure per step
        self.norm_partials = torch.zeros(len(self.buckets), dtype=torch.float32, device=dev)
        # World size 1 on GPU (SFTAMD_NORM_FUSED, default on): the weight-gradient GEMMs of the synchronising pass
        # write the sum of squares of the gradient they store into per-(tile, wave) slots (csrc/gemm_wgrad.hip), so
        # the clip norm is one small reduction over the slots plus a pass over what no wgrad epilogue produced
        # (tied embedding, norm weights, adapters): the 6 GB sum-of-squares pass of a 3B model disappears.
        self.fused_norm = (world_size == 1 and dev.type == "cuda" and not self.track_norm
                           and os.environ.get("SFTAMD_NORM_FUSED", "1") == "1")
        self._norm_slot_views = {}
        self._norm_chunk_cache = {}
        if self.fused_norm:
            total = 0
            offs = []
            for p, _, _, _ in self.layout:
                if p.dim() == 2:
                    cap = -(-p.shape[0] // 256) * -(-p.shape[1] // 128) * 32  # >= slots of any ring launch
                    offs.append((p, total, cap))
                    total += cap
            self.norm_slots = torch.zeros(max(total, 1), dtype=torch.float32, device=dev)
            for p, o, cap in offs:
                self._norm_slot_views[id(p)] = self.norm_slots[o:o + cap]
        self._norm_stream = torch.cuda.Stream(device=dev) if (self.track_norm and dev.type == "cuda") else None
        self._norm_valid = False
        for p, _, _, _ in self.layout:
            p._sftamd_ready_hook = self._on_param_ready
            p.register_post_accumulate_grad_hook(self._post_accumulate)
        if broadcast_params and world_size > 1:
            dist.broadcast(self.param_flat, src=0, group=self.pg)

    # ------------------------------------------------------------------ helpers
    def param_offset(self, p) -> int:
        for q, o, _, _ in self.layout:
            if q is p:
                return o
        raise KeyError

    def params(self):
        return [p for p, _, _, _ in self.layout]

    def named_params(self):
        return [(self.param_names[id(p)], p) for p, _, _, _ in self.layout]

    @torch.no_grad()
    def params_by_name(self) -> torch.Tensor:
        """All trainable parameters concatenated in name order: a world-size-independent view of
        ``param_flat`` (whose bucket padding depends on the world size) for cross-run comparisons."""
        return torch.cat([p.detach().reshape(-1) for _, p in sorted(self.named_params(), key=lambda t: t[0])])

    # ------------------------------------------------------------------ GA / sync control
    @contextlib.contextmanager
    def no_sync(self):
        prev = self.sync_grads
        self.sync_grads = False
        try:
            yield
        finally:
            self.sync_grads = prev

    def zero_grad(self, set_fresh: bool = True):
        """Start a new accumulation window. With ``set_fresh`` (default) no memset is issued: each
        parameter's FIRST gradient contribution overwrites its slice (beta=0 GEMM / copy) and
        ``finish_backward`` zero-fills slices that received nothing (unused parameters)."""
        if not set_fresh:
            self.grad_flat.zero_()
            return
        for p, _, _, _ in self.layout:
            p._sftamd_fresh = True

    def prepare_backward(self):
        """Call before every backward: resets per-parameter use counters and bucket state."""
        self._norm_valid = False
        if self._norm_stream is not None:  # pending norm reads finish before gradients are overwritten
            torch.cuda.current_stream(self.grad_flat.device).wait_stream(self._norm_stream)
        reset = getattr(self.model, "reset_grad_use_counters", None)
        if reset is not None:
            reset()
        self._sparse = None
        if self.tied_param is not None:
            # synchronising pass: the tied weight is complete after its lm_head contribution; the embedding
            # backward hands its sparse rows to _sparse_sink (no_sync passes keep the dense accumulation)
            sparse = self.sync_grads
            self.tied_param._sftamd_sparse_sink = self._sparse_sink if sparse else None
            if sparse:
                self.tied_param._sftamd_remaining = 1
        if self.fused_norm:
            if self.sync_grads:
                self.norm_slots.zero_()
            for p, _, _, _ in self.layout:
                p._sftamd_norm_slots = self._norm_slot_views.get(id(p)) if self.sync_grads else None
                p._sftamd_norm_done = False
        for b in self.buckets:
            b.ready = False
            b.launched = False
            b.work = None
        self.last_launched = -1
        self._tracker.reset()

    # ------------------------------------------------------------------ hooks
    def _zero_untouched(self):
        for p, _, _, _ in self.layout:
            if getattr(p, "_sftamd_fresh", False):
                p.main_grad.zero_()
                p._sftamd_fresh = False

    def _post_accumulate(self, p):
        # Plain-autograd parameters (e.g. LoRA adapters): fold .grad into the flat buffer.
        # The hook also fires for parameters whose fused op returned no gradient (they already
        # accumulated into main_grad and signalled readiness themselves): ignore those, or the
        # bucket would be counted twice and launched before its gradients are complete.
        if p.grad is None:
            return
        if getattr(p, "_sftamd_fresh", False):
            p.main_grad.copy_(p.grad)
            p._sftamd_fresh = False
        else:
            p.main_grad.add_(p.grad.to(p.main_grad.dtype))
        p.grad = None
        self._on_param_ready(p)

    def _on_param_ready(self, p):
        if not self.sync_grads or (self.world_size == 1 and not self.track_norm):
            return
        i = self._param_index.get(id(p))
        if i is None:
            return
        try:
            launch = self._tracker.mark(i)
        except RuntimeError as e:
            raise RuntimeError(f"{e} ({self.param_names.get(id(p))})") from None
        for j in launch:
            self.buckets[j].ready = True
            self._launch(self.buckets[j])

    def bucket_pending(self) -> List[int]:
        """Parameters each bucket still waits for in the current backward (the ready tracker's counts)."""
        return self._tracker.pending()

    def _launch(self, b: Bucket):
        view = self.grad_flat[b.start:b.end]
        ws = None
        if self.world_size > 1:
            self._collective(b, view)
        if self.track_norm:
            self._bucket_norm(b, ws)
        b.launched = True
        self.last_launched = b.index

    def _bucket_norm(self, b: Bucket, ws=None):
        """Sum of squares of bucket ``b``'s reduced gradient (its owned slice under ZeRO-1) into
        ``norm_partials[b.index]``, ordered after the bucket's collective."""
        from ..ops.optim_kernels import sumsq_list
        s, e = self.shard_range(b)
        if e <= s:
            self.norm_partials[b.index].zero_()
            return
        ns = self._norm_stream
        if ns is None:
            if b.work is not None:
                b.work.wait()
            self.norm_partials[b.index].copy_(sumsq_list([self.grad_flat[s:e]]))
            return
        ns.wait_stream(ws if ws is not None else torch.cuda.current_stream(self.grad_flat.device))
        with torch.cuda.stream(ns):
            if b.work is not None:
                b.work.wait()  # the norm stream waits for the collective (no host block)
            self.norm_partials[b.index].copy_(sumsq_list([self.grad_flat[s:e]]))

    def grad_norm_sq(self) -> Optional[torch.Tensor]:
        """This rank's sum of squares of the reduced gradients (owned slices under ZeRO-1), computed during
        the last synchronised backward; None when that backward did not produce it."""
        if not self._norm_valid:
            return None
        if self.fused_norm:
            self._norm_valid = False
            return (self.norm_slots.sum() + self._leftover_sumsq()).reshape(1)
        if self._norm_stream is not None:
            torch.cuda.current_stream(self.grad_flat.device).wait_stream(self._norm_stream)
        self._norm_valid = False
        return self.norm_partials.sum().reshape(1)

    def _leftover_sumsq(self) -> torch.Tensor:
        """Sum of squares of the gradients no wgrad epilogue covered this step, in one launch over
        chunks of grad_flat (256K elements per block; the chunk table is cached per set of leftover ranges)."""
        ranges = []
        for p, o, n, _ in self.layout:
            if not getattr(p, "_sftamd_norm_done", False):
                if ranges and ranges[-1][0] + ranges[-1][1] == o:
                    ranges[-1][1] += n
                else:
                    ranges.append([o, n])
        if not ranges:
            return torch.zeros((), dtype=torch.float32, device=self.grad_flat.device)
        key = tuple((o, n) for o, n in ranges)
        chunks = self._norm_chunk_cache.get(key)
        if chunks is None:
            CH = 1 << 18  # ~1000 blocks for a 262M-element tied embedding
            tab = [(o + s, min(CH, n - s)) for o, n in ranges for s in range(0, n, CH)]
            chunks = torch.tensor(tab, dtype=torch.int64).to(self.grad_flat.device)
            if len(self._norm_chunk_cache) > 16:
                self._norm_chunk_cache.clear()
            self._norm_chunk_cache[key] = chunks
        from ..ops import _ext
        return _ext.ops().sumsq_chunks(self.grad_flat, chunks).sum()

    # ------------------------------------------------------------------ small all-reduces
    def all_reduce_small_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM of a few values (the clip norm): through the peer-memory one-shot kernel
        (parallel/ipc_allreduce.py, one ~10 us launch on the compute stream) when SFTAMD_IPC_ALLREDUCE=1 on GPUs,
        else the process group's all_reduce."""
        if self.world_size == 1:
            return t
        ar = self._small_ar()
        if ar is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= 1024:
            ar.raise_if_failed()  # the previous call's bounded waits (non-blocking read of its error word)
            n = t.numel()
            buf = torch.zeros((n + 3) // 4 * 4, dtype=torch.float32, device=t.device)
            buf[:n].copy_(t.reshape(-1))
            ar.all_reduce_(buf)
            t.copy_(buf[:n].view_as(t))
            return t
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg)
        return t

    def _small_ar(self):
        if not hasattr(self, "_ipc_ar"):
            self._ipc_ar = None
            if (os.environ.get("SFTAMD_IPC_ALLREDUCE", "0") == "1" and self.device.type == "cuda"
                    and self.world_size > 1):
                from .ipc_allreduce import IPCAllReduce
                self._ipc_ar = IPCAllReduce(max_bytes=1 << 16, group=self.pg)
        return self._ipc_ar

    # ------------------------------------------------------------------ sparse tied-embedding gradient
    def _sparse_sink(self, ids: torch.Tensor, rows: torch.Tensor):
        """Embedding backward of the synchronising pass: unique token ids [U] (int64) and their summed gradient
        rows [U, H] (the tied weight's dtype)."""
        self._sparse = (ids, rows)

    def _exchange_sparse(self):
        """All ranks' sparse embedding rows into the (already all-reduced) tied gradient, in rank order: every
        rank computes the same sum (each rank's ids are unique, so every row gets one add per rank; padding slots
        carry id 0 and a zero row, an exact no-op).

        The gather size is the host-known ``sparse_cap`` (the most tokens one synchronising pass can hold, set by
        the trainer from its batch geometry — identical on every rank), so nothing here waits for the device; only
        when no cap is known does it fall back to a MAX all-reduce of the counts plus a host read."""
        p = self.tied_param
        mg = p.main_grad
        H = mg.shape[-1]
        if self._sparse is None:
            ids = torch.empty(0, dtype=torch.int64, device=mg.device)
            rows = torch.empty(0, H, dtype=mg.dtype, device=mg.device)
        else:
            ids, rows = self._sparse
            self.sparse_exchanges += 1
        self._sparse = None
        cap = int(self.sparse_cap or 0)
        if cap <= 0 or ids.numel() > cap:
            if cap > 0:
                raise RuntimeError(f"sparse tied-embedding exchange: {ids.numel()} rows exceed the host cap {cap} "
                                   "(every rank must use the same cap; raise DDPEngine.sparse_cap)")
            n = torch.tensor([ids.numel()], dtype=torch.int64, device=mg.device)
            dist.all_reduce(n, op=dist.ReduceOp.MAX, group=self.pg)
            cap = max(1, int(n.item()))
        if ids.numel() == cap:
            idp, rwp = ids, rows
        else:
            idp = torch.zeros(cap, dtype=torch.int64, device=mg.device)  # padding -> row 0, with zero rows
            rwp = torch.zeros(cap, H, dtype=mg.dtype, device=mg.device)
            idp[:ids.numel()] = ids
            rwp[:ids.numel()] = rows
        gid = torch.empty(self.world_size * cap, dtype=torch.int64, device=mg.device)
        grw = torch.empty(self.world_size * cap, H, dtype=mg.dtype, device=mg.device)
        dist.all_gather_into_tensor(gid, idp.contiguous(), group=self.pg)
        dist.all_gather_into_tensor(grw, rwp.contiguous(), group=self.pg)
        for r in range(self.world_size):
            mg.index_add_(0, gid[r * cap:(r + 1) * cap], grw[r * cap:(r + 1) * cap])

    def _collective(self, b: Bucket, view: torch.Tensor):
        if self.shard and not b.replicated:
            s, e = self.shard_range(b)
            # in place: this rank's slice of the bucket receives the sum of every rank's slice
            b.work = dist.reduce_scatter_tensor(self.grad_flat[s:e], view, op=dist.ReduceOp.SUM, group=self.pg,
                                                async_op=True)
        else:
            b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    # ------------------------------------------------------------------ ZeRO-1 slices
    def shard_range(self, b: Bucket):
        """[start, end) of the slice of bucket ``b`` this rank owns (the whole bucket unless sharded)."""
        if not self.shard or self.world_size == 1 or b.replicated:
            return b.start, b.end
        n = (b.end - b.start) // self.world_size
        return b.start + self.rank * n, b.start + (self.rank + 1) * n

    def owned_ranges(self):
        return [self.shard_range(b) for b in self.buckets]

    def gather_params(self, b: Bucket, async_op: bool = True):
        """All-gather the updated parameter slices of bucket ``b`` (in place) — ZeRO-1 only."""
        if not self.shard or self.world_size == 1 or b.replicated:
            return None
        s, e = self.shard_range(b)
        return dist.all_gather_into_tensor(self.param_flat[b.start:b.end], self.param_flat[s:e], group=self.pg,
                                           async_op=async_op)

    def finish_backward(self):
        """Wait for all bucket all-reduces (launching any bucket whose params had no grad)."""
        if not self.sync_grads:
            return
        self._zero_untouched()
        if self.fused_norm:
            self._norm_valid = True
        if self.world_size == 1 and not self.track_norm:
            return
        for j in self._tracker.drain():
            self._launch(self.buckets[j])
        self._norm_valid = self.track_norm
        if self.world_size == 1:
            return
        timing = self.grad_flat.is_cuda
        if timing:  # exposed communication = what the compute stream waits for after its last kernel
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
        if self.tied_param is not None:
            self._exchange_sparse()
        if timing:
            e1.record()
            self._comm_events.append((e0, e1))
            if len(self._comm_events) > 64:  # bounded when nobody reads them (e.g. logging off)
                del self._comm_events[0]

    def comm_exposed_ms(self, reset: bool = True) -> float:
        """Mean exposed (non-overlapped) gradient-communication time per synchronised backward, in ms,
        since the last call (reads CUDA events: call at log time, not per step)."""
        ev = self._comm_events
        if not ev:
            return 0.0
        ev[-1][1].synchronize()
        v = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        if reset:
            self._comm_events = []
        return v

    # ------------------------------------------------------------------ debug / safety
    @torch.no_grad()
    def param_checksum(self) -> torch.Tensor:
        return self.param_flat.float().sum().reshape(1)

    @torch.no_grad()
    def assert_in_sync(self, tol: float = 0.0):
        """Cross-rank parameter checksum (catches DDP desync)."""
        if self.world_size == 1:
            return
        c = self.param_checksum()
        lst = [torch.zeros_like(c) for _ in range(self.world_size)]
        dist.all_gather(lst, c, group=self.pg)
        vals = torch.cat(lst)
        if (vals - vals[0]).abs().max().item() > tol * max(1.0, vals[0].abs().item()):
            raise RuntimeError(f"DDP desync: parameter checksums differ across ranks: {vals.tolist()}")
