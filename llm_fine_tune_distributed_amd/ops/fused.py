"""Autograd Functions for the SmolLM3/Llama hot path.

Every Function is device-agnostic: on GPU tensors it calls the CDNA4 HIP kernels in
``torch.ops.sftamd`` (csrc/*.hip); on CPU tensors it runs ``ops.reference``. The same
gradient plumbing runs in both cases, so CPU tests exercise it.

Gradient plumbing (replaces the c10d Reducer's copy-into-bucket):
trainable parameters may carry ``param.main_grad`` — a view into the DDP engine's flat,
bucketed gradient buffer. Weight gradients are accumulated *directly* into it (GEMM with
beta=1 for linears, fused reductions for norms, a deterministic segment-sum for the
embedding), and autograd never materialises ``param.grad``. Each parameter declares how
many times it is used per forward (``_sftamd_uses``; 2 for a tied embedding); when all
uses have been back-propagated the parameter's ready-hook fires, which is what lets the
DDP engine launch bucket all-reduces while backward is still running.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Optional, Tuple

import torch
from torch.autograd import Function

from . import _ext
from . import reference as ref

IGNORE_INDEX = -100


# ----------------------------------------------------------------------------- grad plumbing
def _weight_grad_done(param: torch.Tensor) -> None:
    rem = getattr(param, "_sftamd_remaining", None)
    if rem is None:
        return
    rem -= 1
    param._sftamd_remaining = rem
    if rem <= 0:
        hook = getattr(param, "_sftamd_ready_hook", None)
        if hook is not None:
            hook(param)


_WGRAD_MODE = os.environ.get("SFTAMD_WGRAD", "auto")  # auto | blas | <cfg int> (kernel variant)


_NUM_CUS = 256  # MI355X: 8 XCDs x 32 CUs


def _budget_from_env() -> int:
    try:
        b = int(os.environ.get("SFTAMD_CU_BUDGET", "0") or 0)
    except ValueError:
        b = 0
    return b if 0 < b < _NUM_CUS else _NUM_CUS


_CU_BUDGET = _budget_from_env()  # the C++ side reads the same variable (csrc/cu_budget.h)


def set_cu_budget(n: int) -> int:
    """The CU count the one-round GEMM grids are sized for (0 = all 256). When collectives overlap compute at N > 1,
    RCCL's channel blocks hold some CUs and a grid of exactly 256 one-per-CU workgroups waits a second round for
    them (sftamd.cu_hog measurements, profiles/r6_cu_contention.md); with a budget the split / hybrid decisions of
    the 4-wave GEMMs (here and in csrc/gemm_4w.hip) leave that many CUs free. Returns the effective budget."""
    global _CU_BUDGET
    b = int(n) if 0 < int(n) < _NUM_CUS else _NUM_CUS
    if _ext.load():
        b = int(_ext.ops().set_cu_budget(0 if b == _NUM_CUS else b))
    _CU_BUDGET = b
    return b


def cu_budget() -> int:
    return _CU_BUDGET


def _wgrad_cfg(T: int, N: int, K: int) -> int:
    """Which wgrad GEMM runs dW[N,K] = dy[T,N]^T x[T,K]: 0 = hipBLASLt/rocBLAS, else a csrc/gemm_wgrad.hip cfg
    (1000 H + 100 S + c). From interleaved A/Bs on MI355X at T = 8192 (tools/bench_ab.py, profiles/r6_gemm_routing.md):
    the 4-wave ring with one read / DMA piece per MFMA gap (c = 14, csrc/gemm_4w.hip) on every shape with N, K % 256 and
    T % 128 — small grids split over the tokens so they fill the chip (qkv 96 tiles x 2: 0.1025 vs 0.1155 ms for the
    pair-loop kernel; o_proj 64 tiles x 4: 0.0705 vs 0.0715 for the 8-wave 256 x 128 ring split 2), grids whose last
    round is partial hybrid-split (down_proj 344 tiles: 0.274 vs 0.310 unsplit; lm_head 4008: 2.969 vs 3.237 for the
    8-wave 256 x 256 ring), gate_up (688 tiles) unsplit (0.534 vs 0.575 hybrid). Stream-K over the last round was
    no faster on any of them. The 8-wave rings (c = 9 / 10) remain for K % 256 != 0 or T % 128 != 0."""
    if _WGRAD_MODE == "blas" or T % 32 or T < 1024:
        return 0
    if _WGRAD_MODE not in ("auto", ""):
        return int(_WGRAD_MODE)
    tiles = (N // 256) * (K // 256)
    B = _CU_BUDGET  # one round of workgroups (256 unless collectives hold CUs: set_cu_budget)
    if N % 256 == 0 and K % 256 == 0 and T % 128 == 0:
        if tiles < B:
            s = min(8, B // tiles, T // 128)
            return 100 * s + 14 if s >= 2 else 14
        if (tiles < 2 * B or tiles >= 8 * B) and tiles % B and T // 128 >= 2:
            return 1214
        return 14
    if N % 256 == 0 and K % 256 == 0 and tiles >= 512:
        return 10
    if (N % 256 == 0 and K % 256 == 0 and 64 < tiles <= 128 and (T // 32) % 2 == 0
            and (N // 256) * (K // 128) < 256):
        return 210
    if N % 256 == 0 and K % 128 == 0 and (N // 256) * (K // 128) >= 160:
        return 9
    if N % 256 == 0 and K % 128 == 0 and (T // 32) % 2 == 0 and (N // 256) * (K // 128) >= 32:
        return 209
    return 0


def _wgrad_mm(out: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor, accumulate: bool,
              norm: Optional[torch.Tensor] = None) -> bool:
    """out (+)= dy2d^T @ x2d, all bf16 (out is the flat-buffer gradient view). ``norm``: gradient-norm partial
    slots the ring kernels fill with the sum of squares of the values they store; returns whether they did
    (other variants leave the norm to DDPEngine.grad_norm_sq's leftover pass)."""
    cfg = 0
    if _ext.use_hip(dy2d) and dy2d.dtype == torch.bfloat16 and out.is_contiguous():
        cfg = _wgrad_cfg(dy2d.shape[0], dy2d.shape[1], x2d.shape[1])
    if cfg:
        use_norm = norm is not None and cfg % 100 in (9, 10, 14)
        # the 4-wave kernel reads x through its row pitch (a padded [T, K] view, e.g. the gate_up input); others copy
        strided_ok = cfg % 100 == 14 and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0 and x2d.data_ptr() % 16 == 0
        _ext.ops().wgrad_gemm(out, dy2d.contiguous(), x2d if strided_ok else x2d.contiguous(), accumulate, cfg,
                              norm if use_norm else None)
        return use_norm
    if accumulate:
        out.addmm_(dy2d.t(), x2d)
    else:
        torch.mm(dy2d.t(), x2d, out=out)
    return False


def _accumulate_weight_grad(param: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor,
                            scale: Optional[torch.Tensor] = None):
    """dW = dy^T @ x (optionally * scale). Accumulates into main_grad if present."""
    mg = getattr(param, "main_grad", None)
    if scale is not None:
        x2d = x2d * scale.to(x2d.dtype)
    if mg is not None:
        fresh = getattr(param, "_sftamd_fresh", False)
        if mg.dtype == dy2d.dtype:
            # first contribution of the step: beta=0 GEMM, no zero-fill pass needed. Norm partials (DDPEngine
            # fused norm, synchronising pass only) when this is the parameter's last contribution of the pass.
            ns = getattr(param, "_sftamd_norm_slots", None)
            if ns is not None and getattr(param, "_sftamd_remaining", 1) != 1:
                ns = None
            done = _wgrad_mm(mg, dy2d, x2d, accumulate=not fresh, norm=ns)
            if done:
                param._sftamd_norm_done = True
        elif fresh:
            mg.copy_(torch.mm(dy2d.t(), x2d))
        else:
            mg.add_(torch.mm(dy2d.t(), x2d).to(mg.dtype))
        param._sftamd_fresh = False
        _weight_grad_done(param)
        return None
    return torch.mm(dy2d.t(), x2d).to(param.dtype)


# Weight gradients in pairs as ONE 4-wave grid: the MLP's down projection defers its weight gradient to the gate_up
# node, the attention's o_proj to the qkv + RoPE + attention node (per-call dicts link them), which then issue both in
# one launch — MLP: 344 + 688 tiles = 4.03 rounds of 256 CUs instead of 1.34 + 2.69 with a partial last round each (a
# partial round costs 0.75-1 of a full one: tools/debug/round_scaling.py, profiles/r6_gemm_routing.md); attention:
# 64 + 96 tiles split 3 ways = 2 rounds of third-tiles. SFTAMD_WGRAD_PAIR=0: off.
_WGRAD_PAIR = os.environ.get("SFTAMD_WGRAD_PAIR", "1") == "1"


def _job_ok(p, dy, x) -> bool:
    """A weight gradient the 4-wave multi-problem launches take (bf16 main_grad, 256-multiple shapes, aligned rows)."""
    mg = getattr(p, "main_grad", None)
    return (mg is not None and mg.dtype == torch.bfloat16 and mg.is_contiguous() and dy.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16 and dy.shape[1] % 256 == 0 and x.shape[1] % 256 == 0
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and dy.data_ptr() % 16 == 0
            and mg.data_ptr() % 16 == 0)


def _pair_ok(p0, dy0, x0, p1, dy1, x1) -> bool:
    one = _job_ok
    if not (_WGRAD_PAIR and _WGRAD_MODE in ("auto", "") and dy0.is_cuda and _ext.use_hip(dy0)):
        return False
    T = dy0.shape[0]
    if not (T % 128 == 0 and T >= 1024 and dy1.shape[0] == T and x0.shape[0] == T and x1.shape[0] == T):
        return False
    if not (one(p0, dy0, x0) and one(p1, dy1, x1)):
        return False
    t0 = (dy0.shape[1] // 256) * (x0.shape[1] // 256)
    t1 = (dy1.shape[1] // 256) * (x1.shape[1] // 256)
    return _pair_split(t0, t1, T) > 1 or (t0 + t1) % _CU_BUDGET <= t1


def _pair_split(t0: int, t1: int, T: int) -> int:
    """Pairs smaller than one round (o_proj + qkv: 64 + 96 tiles) split every tile s ways, s minimising the rounds of
    1/s-tiles plus the fp32 slab traffic of the fixup (~4e-4 of a tile's time per piece at T = 8192, from the o_proj /
    qkv split launches: profiles/r6_gemm_routing.md) — 3 for o_proj + qkv (480 pieces = 2 rounds of third-tiles);
    0 = whole rounds + the split leftover (hybrid)."""
    n = t0 + t1
    if n >= _CU_BUDGET:
        return 0
    best, cost = 0, None
    for s in range(2, min(8, T // 128) + 1):
        c = -(-n * s // _CU_BUDGET) / s + 4e-4 * n * s
        if cost is None or c < cost - 1e-9:
            best, cost = s, c
    return best


def _accumulate_weight_grad_pair(p0, dy0, x0, p1, dy1, x1):
    """_accumulate_weight_grad(p0, dy0, x0) and (p1, dy1, x1) — one wgrad_gemm_pair launch where it applies."""
    if not _pair_ok(p0, dy0, x0, p1, dy1, x1):
        _accumulate_weight_grad(p0, dy0, x0)
        _accumulate_weight_grad(p1, dy1, x1)
        return
    split_all = _pair_split((dy0.shape[1] // 256) * (x0.shape[1] // 256), (dy1.shape[1] // 256) * (x1.shape[1] // 256),
                            dy0.shape[0])

    def slots(p):
        ns = getattr(p, "_sftamd_norm_slots", None)
        return ns if (ns is not None and getattr(p, "_sftamd_remaining", 1) == 1) else None

    n0, n1 = slots(p0), slots(p1)
    _ext.ops().wgrad_gemm_pair(p0.main_grad, dy0.contiguous(), x0, not getattr(p0, "_sftamd_fresh", False), n0,
                               p1.main_grad, dy1.contiguous(), x1, not getattr(p1, "_sftamd_fresh", False), n1,
                               split_all)
    for p, ns in ((p0, n0), (p1, n1)):
        if ns is not None:
            p._sftamd_norm_done = True
        p._sftamd_fresh = False
        _weight_grad_done(p)


# SFTAMD_WGRAD_CARRY=0: a layer's o_proj + qkv weight gradients launch on their own (2 rounds of third-tiles)
# instead of joining the previous layer's down + gate_up launch
_WGRAD_CARRY = os.environ.get("SFTAMD_WGRAD_CARRY", "1") == "1"


def _multi_split(total: int, T: int) -> int:
    """Ways to split the partial last round of a multi-problem launch over the tokens: the count minimising the rounds
    of 1/s-tiles plus the fp32 slab traffic (the cost model of _pair_split); 1 = no split. An unsplit partial round
    costs at least 0.75 of a full one (tools/debug/round_scaling.py) — and no slabs: the SmolLM3 layer grid (1192
    tiles, 168 left over) measured 0.9185 ms unsplit vs 0.9325 split 3 ways, 0.9466 / 0.9558 for 2 / 4
    (tools/bench_pair.py --pair layer, profiles/r6_gemm_routing.md)."""
    left = total % _CU_BUDGET
    if left == 0:
        return 1
    forced = os.environ.get("SFTAMD_MULTI_SPLIT", "")
    if forced:
        return max(1, int(forced))
    best, cost = 1, max(0.75, left / _CU_BUDGET)
    for s in range(2, min(8, T // 128) + 1):
        c = -(-left * s // _CU_BUDGET) / s + 4e-4 * left * s
        if c < cost - 1e-9:
            best, cost = s, c
    return best


def _multi_ok(jobs) -> bool:
    p0, dy0, x0 = jobs[0]
    if not (_WGRAD_PAIR and _WGRAD_MODE in ("auto", "") and dy0.is_cuda and _ext.use_hip(dy0)):
        return False
    T = dy0.shape[0]
    if not (T % 128 == 0 and T >= 1024 and all(dy.shape[0] == T and x.shape[0] == T for _, dy, x in jobs)):
        return False
    if not all(_job_ok(p, dy, x) for p, dy, x in jobs):
        return False
    return sum((dy.shape[1] // 256) * (x.shape[1] // 256) for _, dy, x in jobs) >= _CU_BUDGET


def _accumulate_weight_grad_jobs(jobs):
    """Weight gradients [(param, dy2d, x2d)] over the same tokens: ONE wgrad_gemm_multi launch for 3-4 of them (a
    layer's down + gate_up with the next layer's o_proj + qkv: 1192 tiles = 4 whole rounds + a partial round of 168
    tiles, against 4 rounds + 8 split tiles and a separate 2-round grid of third-tiles), pairs / single launches otherwise."""
    if len(jobs) == 1:
        _accumulate_weight_grad(*jobs[0])
        return
    if len(jobs) == 2:
        _accumulate_weight_grad_pair(*jobs[0], *jobs[1])
        return
    if not _multi_ok(jobs):
        _accumulate_weight_grad_jobs(jobs[:2])
        _accumulate_weight_grad_jobs(jobs[2:])
        return
    T = jobs[0][1].shape[0]
    total = sum((dy.shape[1] // 256) * (x.shape[1] // 256) for _, dy, x in jobs)
    split_left = _multi_split(total, T)

    def slots(p):
        ns = getattr(p, "_sftamd_norm_slots", None)
        return ns if (ns is not None and getattr(p, "_sftamd_remaining", 1) == 1) else None

    ns = [slots(p) for p, _, _ in jobs]
    empty = jobs[0][1].new_empty(0, dtype=torch.float32)
    _ext.ops().wgrad_gemm_multi([p.main_grad for p, _, _ in jobs], [dy.contiguous() for _, dy, _ in jobs],
                                [x for _, _, x in jobs], [0 if getattr(p, "_sftamd_fresh", False) else 1 for p, _, _ in jobs],
                                [n if n is not None else empty for n in ns], 0, split_left)
    for (p, _, _), n in zip(jobs, ns):
        if n is not None:
            p._sftamd_norm_done = True
        p._sftamd_fresh = False
        _weight_grad_done(p)


# The hand-off of a layer's attention weight gradients to the previous layer's MLP launch: CausalLM.forward opens a
# scope; swiglu_mlp leaves its (armed) dict in it and the next layer's attention node takes that dict, deposits its
# o_proj + qkv weight-gradient jobs there in its backward (which always runs before the previous layer's gate_up
# backward: that node's output feeds this layer), and the gate_up node launches all four at once.
_CARRY = None


class wgrad_carry_scope:
    """`with wgrad_carry_scope(enabled):` around the decoder-layer loop of one forward (no activation checkpointing:
    recomputed layers would arm dicts whose nodes never run)."""

    def __init__(self, enabled: bool = True):
        self.enabled = bool(enabled and _WGRAD_CARRY and _WGRAD_PAIR and torch.is_grad_enabled())

    def __enter__(self):
        global _CARRY
        self.prev = _CARRY
        _CARRY = {"mlp": None} if self.enabled else None
        return self

    def __exit__(self, *exc):
        global _CARRY
        _CARRY = self.prev
        return False


def _carry_put(box: Optional[dict]) -> None:
    if _CARRY is not None:
        _CARRY["mlp"] = box if (box is not None and box.get("armed")) else None


def _carry_take() -> Optional[dict]:
    if _CARRY is None:
        return None
    box, _CARRY["mlp"] = _CARRY["mlp"], None
    return box


def _carry_or_launch(carry: Optional[dict], jobs) -> None:
    """The attention node's weight-gradient jobs: into the previous layer's MLP dict when it will launch them with its
    own (armed, 4-problem launch eligible), else now."""
    if (carry is not None and carry.get("armed") and "attn" not in carry and len(jobs) == 2
            and all(getattr(p, "main_grad", None) is not None for p, _, _ in jobs)):
        carry["attn"] = jobs
        return
    _accumulate_weight_grad_jobs(jobs)


def _accumulate_small_grad(param: torch.Tensor, g: torch.Tensor):
    mg = getattr(param, "main_grad", None)
    if mg is not None:
        if getattr(param, "_sftamd_fresh", False):
            mg.copy_(g)
            param._sftamd_fresh = False
        else:
            mg.add_(g.to(mg.dtype))
        _weight_grad_done(param)
        return None
    return g.to(param.dtype)


# ----------------------------------------------------------------------------- forward GEMMs
# The plain projection forwards (o_proj, down_proj, lm_head, NoPE-layer qkv) are plain library GEMMs with nothing to
# fuse: hipBLASLt (TunableOp selections). The hand-written persistent 4-wave kernel lost to it end to end by 3-5 %
# (static, per-tile and work-stealing launches, with and without the overlapped AdamW: profiles/r4_gemm_fwd.md); the
# hand-written forward GEMMs keep the fused epilogues — qkv + RoPE, the optional gate_up + SwiGLU, the LoRA wide GEMM.


def _as_output(y2d: torch.Tensor, lead) -> torch.Tensor:
    """[M, N] GEMM result -> [*lead, N] returned from a custom Function forward WITHOUT view semantics (the result
    is an intermediate of the Function; a .view() of it would make in-place consumers such as rope_ fail autograd's
    view + in-place check)."""
    shape = (*lead, y2d.shape[-1])
    return y2d if tuple(y2d.shape) == shape else torch.ops.aten._unsafe_view(y2d, shape)


# Plain projection forwards: hipBLASLt where TunableOp holds a measured selection for the exact shape (the bench's
# 16 x 512 tokens: it stays 1 % ahead of the hand-written kernel in the step), the row-contiguous persistent kernel
# everywhere else — the ragged padding-free batches of real data (M ~ 10k, a new M almost every step) and eval batches,
# where hipBLASLt's default heuristics pick split-K kernels that took 36 % of the recipe's kernel time
# (profiles/r5_recipe.md). SFTAMD_FWD_GEMM: auto (this rule) | blas | hip.
_FWD_GEMM = os.environ.get("SFTAMD_FWD_GEMM", "auto")
_ROWC_CFG = int(os.environ.get("SFTAMD_TN_CFG", "60"))  # row-contiguous persistent kernel (60: cacheable stores)


def _rowc_ok(x2d: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the row-contiguous persistent forward GEMM (csrc/gemm_tn.hip cfg 60 / 61) takes."""
    M, K = x2d.shape
    return (_ext.use_hip(x2d) and x2d.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and M % 256 == 0
            and M > 0 and K % 128 == 0 and w.shape[0] % 256 == 0 and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0
            and w.is_contiguous() and x2d.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def _fwd_on_hip(x2d: torch.Tensor, w: torch.Tensor) -> bool:
    if _FWD_GEMM == "blas" or not _rowc_ok(x2d, w):
        return False
    if _FWD_GEMM == "hip":
        return True
    from ..utils.gemm_tuning import tuned_tn_shapes
    return (w.shape[0], x2d.shape[0], x2d.shape[1]) not in tuned_tn_shapes() or x2d.stride(0) != x2d.shape[1]


def fwd_gemm(x2d: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x2d @ w^T for a plain projection forward: hipBLASLt for shapes with a TunableOp selection, the
    row-contiguous HIP kernel (csrc/gemm_tn.hip tn6) otherwise (see _FWD_GEMM)."""
    if _fwd_on_hip(x2d, w):
        return _ext.ops().gemm_tn(x2d, w, _ROWC_CFG)
    return torch.nn.functional.linear(x2d, w)


# ----------------------------------------------------------------------------- linear
class LinearFn(Function):
    @staticmethod
    def forward(ctx, x, weight):
        ctx.save_for_backward(x)
        ctx.weight = weight
        x2d = x.reshape(-1, x.shape[-1])
        if _ext.use_hip(x2d):
            return _as_output(fwd_gemm(x2d, weight), x.shape[:-1])
        return torch.nn.functional.linear(x, weight)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad_mm(dy2d, w).view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dy2d, x.reshape(-1, x.shape[-1]))
        return dx, dw


def linear(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    return LinearFn.apply(x, weight)


class PairedLinearFn(Function):
    """y = x W^T (LinearFn) for a projection whose CONSUMER defers its own weight gradient here through `box[key]`:
    the MLP's gate_up (the down projection, SwiGLULinearFn, leaves "down") and a NoPE layer's qkv (o_proj,
    AttnOutLinearFn, leaves "o_wgrad"). The backward issues both weight gradients as one launch
    (_accumulate_weight_grad_pair) after this node's input gradient."""

    @staticmethod
    def forward(ctx, x, weight, box, key, arm, carry=None):
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.box = box
        ctx.key = key
        ctx.carry = carry
        if weight.requires_grad:  # this node's backward will run: the consumer may leave its weight gradient to it
            box[arm] = True
        x2d = x.reshape(-1, x.shape[-1])
        return _as_output(fwd_gemm(x2d, weight), x.shape[:-1])

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1])
        x2d = x.reshape(-1, x.shape[-1])
        pending = ctx.box.pop(ctx.key, None)
        extra = ctx.box.pop("attn", None)  # the next layer's o_proj + qkv jobs (_carry_or_launch)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad_mm(dy2d, w).view(*dy.shape[:-1], w.shape[1])
        jobs = [pending] if pending is not None else []
        if ctx.needs_input_grad[1] and getattr(w, "main_grad", None) is not None:
            jobs.append((w, dy2d, x2d))
        elif ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dy2d, x2d)
        if ctx.carry is not None and ctx.key == "o_wgrad":  # a NoPE layer's qkv: the previous layer's MLP may take them
            if jobs:
                _carry_or_launch(ctx.carry, jobs)
        else:
            if jobs:
                _accumulate_weight_grad_jobs(jobs + (extra or []))
            elif extra:
                _accumulate_weight_grad_jobs(extra)
        return dx, dw, None, None, None, None


def mlp_in_linear(x: torch.Tensor, weight: torch.Tensor, box: Optional[dict]) -> torch.Tensor:
    """gate_up(x) whose backward also issues the down projection's weight gradient (swiglu_linear with `box`)."""
    if box is not None and _ext.use_hip(x):
        return PairedLinearFn.apply(x, weight, box, "down", "armed")
    return LinearFn.apply(x, weight)


def qkv_in_linear(x: torch.Tensor, weight: torch.Tensor, box: Optional[dict]) -> torch.Tensor:
    """qkv(x) of a NoPE layer whose backward also issues o_proj's weight gradient (attn_out_linear with `box`) — or
    hands both to the previous layer's MLP launch (wgrad_carry_scope)."""
    if box is not None and _WGRAD_PAIR and _ext.use_hip(x):
        return PairedLinearFn.apply(x, weight, box, "o_wgrad", "wgrad_pair", _carry_take())
    return LinearFn.apply(x, weight)


def _delta_ok(dy2d: torch.Tensor, w: torch.Tensor, a2d: torch.Tensor) -> bool:
    """Shapes dgrad_gemm_delta takes: the 4-wave dgrad (cfg 14) without split-K, a [M, N] attention output with
    16-byte aligned rows, head_dim 128 (N % 256)."""
    M, K = dy2d.shape
    tiles = (M // 256) * (w.shape[1] // 256)
    # (under a reduced CU budget a partial last round is split over K, which the delta epilogue cannot take: the
    # attention node's own delta kernel is cheaper than a second round of whole tiles)
    return (_dgrad_ok(dy2d, w) and K % 128 == 0 and K < 8192 and a2d.dtype == torch.bfloat16
            and (_CU_BUDGET >= _NUM_CUS or tiles % _CU_BUDGET == 0 or tiles < _CU_BUDGET)
            and a2d.shape == (M, w.shape[1]) and a2d.stride(1) == 1 and a2d.stride(0) % 8 == 0
            and a2d.data_ptr() % 16 == 0)


class AttnOutLinearFn(Function):
    """The attention output projection y = a W_o^T behind a fused attention node (QKVRopeAttnFn / FlashAttnFn). Its
    backward computes dO = dy W_o on the 4-wave kernel with flash attention's delta = rowsum(dO . a) per head in the
    epilogue (dgrad_gemm_delta: `a` is this node's saved input, the attention output) and leaves it in `box` for the
    attention node, whose backward then skips its delta kernel (a full re-read of dO and O, ~13 us per layer at
    16 x 512). The attention node checks that the gradient it receives IS that dO (same storage) before using it."""

    @staticmethod
    def forward(ctx, x, weight, box):
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.box = box
        x2d = x.reshape(-1, x.shape[-1])
        return _as_output(fwd_gemm(x2d, weight), x.shape[:-1])

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1])
        x2d = x.reshape(-1, x.shape[-1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if ctx.box.get("armed") and _delta_ok(dy2d, w, x2d):
                d2d, delta = _ext.ops().dgrad_gemm_delta(dy2d, w, x2d)
                ctx.box["delta"] = (delta, d2d.data_ptr(), d2d.shape)
            else:
                d2d = dgrad_mm(dy2d, w)
            dx = d2d.view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            if ctx.box.get("wgrad_pair") and getattr(w, "main_grad", None) is not None:
                ctx.box["o_wgrad"] = (w, dy2d, x2d)  # issued with qkv's (QKVRopeAttnFn.backward)
            else:
                dw = _accumulate_weight_grad(w, dy2d, x2d)
        return dx, dw, None


# SFTAMD_ATTN_DELTA=0: the attention node computes its own delta (delta kernel); also a test seam
_DELTA_FUSED = os.environ.get("SFTAMD_ATTN_DELTA", "1") != "0"


def attn_out_linear(a: torch.Tensor, weight: torch.Tensor, box: Optional[dict]) -> torch.Tensor:
    """o_proj(a) for `a` from qkv_rope_attention / flash_attention called with the same `box` (a fresh dict per
    layer call): the delta hand-off above when the HIP paths apply, linear() otherwise."""
    if _DELTA_FUSED and box is not None and box.get("armed") and _ext.use_hip(a):
        return AttnOutLinearFn.apply(a, weight, box)
    return LinearFn.apply(a, weight)


def _take_delta(box: Optional[dict], dout: torch.Tensor, n_q: int):
    """The delta AttnOutLinearFn left for this attention node, if the incoming gradient is the dO it computed it for
    (the same storage and shape: no other consumer of the attention output added into it)."""
    if box is None:
        return None
    got = box.pop("delta", None)
    if got is None:
        return None
    delta, ptr, shape = got
    if dout.data_ptr() != ptr or dout.reshape(-1, dout.shape[-1]).shape != shape or not dout.is_contiguous():
        return None
    if delta.shape != (n_q, shape[0]):
        return None
    return delta


# ----------------------------------------------------------------------------- input-gradient GEMM
_DGRAD_MODE = os.environ.get("SFTAMD_DGRAD", "auto")  # auto | blas | hip


def _dgrad_ok(dy2d: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the hand-written NN dgrad (csrc/gemm_dgrad.hip, 256 x 256 tiles) handles."""
    M, K = dy2d.shape
    N = w.shape[1]
    return (_DGRAD_MODE != "blas" and _ext.use_hip(dy2d) and dy2d.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and M % 256 == 0 and M > 0 and N % 256 == 0 and K % 32 == 0 and dy2d.stride(1) == 1 and w.stride(1) == 1
            and dy2d.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and dy2d.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0)


# SFTAMD_DGRAD_RING8=0: plain dgrads stay on the 4-wave ring (cfg 14) whatever the grid; also the A/B seam
_DGRAD_RING8 = os.environ.get("SFTAMD_DGRAD_RING8", "1") != "0"


def _ring8_rounds(M: int, N: int) -> bool:
    """The 8-wave rings run whole rounds of 256 x 256 tiles over the 256 CUs, or the wave-tail launch of
    dgrad_gemm (csrc/gemm_dgrad.hip) turns the partial last round into one round of 256 x 128 half tiles."""
    nbm, nbn = M // 256, N // 256
    tiles = nbm * nbn
    if tiles % _NUM_CUS == 0:
        return True
    if tiles < _NUM_CUS or _NUM_CUS % nbm:
        return False
    main_n = tiles // _NUM_CUS * (_NUM_CUS // nbm)
    return (nbn - main_n) * (M // 128) <= _NUM_CUS


def _dgrad_cfg(dy2d: torch.Tensor, swiglu: bool = False, N: Optional[int] = None) -> int:
    """Kernel configuration (csrc/gemm_dgrad.hip). 5 = the 8-wave 32-deep three-stage ring, 7 = its 64-deep
    two-stage sibling, both with conflict-free natural-order transposed reads; 14 = the 4-wave ring of
    csrc/gemm_4w.hip (one read / DMA piece per MFMA gap, split-K for a partial last round).
    M = 8192 (profiles/r6_gemm_routing.md, interleaved, ms): SwiGLU-fused down 0.400 (5) vs 0.409 (7) vs 0.483
    (4-wave register epilogue); plain gate_up 0.535 (5) vs 0.546 (14), down 0.289 vs 0.297, qkv 0.0789 vs 0.0788,
    o 0.058 vs 0.0597, lm_head 3.11 vs 3.04 -> cfg 5 when its grid is whole rounds (or the wave tail applies) and
    the reduction is not vocabulary-long, cfg 14 otherwise (ragged token counts: its split-K tail)."""
    K = dy2d.shape[1]
    if swiglu:
        return 5
    if K % 128 == 0:
        if (_DGRAD_RING8 and N is not None and K < 65536 and _ring8_rounds(dy2d.shape[0], N)):
            return 5
        return 14
    return 7 if K % 64 == 0 else 5


def dgrad_mm(dy2d: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dy @ W (W = the projection's [out, in] weight). The HIP kernel where it beats hipBLASLt: every
    SmolLM3 / Llama shape with M % 256 == 0 and K % 128 == 0 (gate_up and lm_head included; cfg 5 or 14,
    _dgrad_cfg); reductions that are not a multiple of 128 of at most 4096 output features into at most 4096 inputs
    on cfg 7 / 5."""
    if _dgrad_ok(dy2d, w):
        cfg = _dgrad_cfg(dy2d, N=w.shape[1])
        if dy2d.shape[1] % 128 == 0 or _DGRAD_MODE == "hip" or (dy2d.shape[1] <= 4096 and w.shape[1] <= 4096):
            return _ext.ops().dgrad_gemm(dy2d, w, None, cfg)
    return torch.mm(dy2d, w)


class SwiGLULinearFn(Function):
    """y = swiglu(gu) @ W^T — the MLP down projection with its SwiGLU input. Backward: ONE
    HIP GEMM dgu = swiglu_bwd(dy @ W, gu) with the SwiGLU backward in the epilogue (the [M, I] dact is never
    written), plus the weight gradient from the saved activation."""

    @staticmethod
    def forward(ctx, gu, weight, box=None):
        act = _ext.ops().swiglu_fwd(gu)
        ctx.save_for_backward(gu, act)
        ctx.weight = weight
        ctx.box = box
        a2d = act.reshape(-1, act.shape[-1])
        return _as_output(fwd_gemm(a2d, weight), gu.shape[:-1])

    @staticmethod
    def backward(ctx, dy):
        gu, act = ctx.saved_tensors
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1]).contiguous()
        gu2d = gu.reshape(-1, gu.shape[-1])
        dgu = dw = None
        if ctx.needs_input_grad[0]:
            if _dgrad_ok(dy2d, w) and gu2d.is_contiguous():
                dgu = _ext.ops().dgrad_gemm(dy2d, w, gu2d, _dgrad_cfg(dy2d, swiglu=True))
            else:
                dgu = _ext.ops().swiglu_bwd(torch.mm(dy2d, w), gu2d)
            dgu = dgu.view(gu.shape)
        if ctx.needs_input_grad[1]:
            a2d = act.reshape(-1, act.shape[-1])
            box = ctx.box
            if box is not None and box.get("armed") and getattr(w, "main_grad", None) is not None:
                box["down"] = (w, dy2d, a2d)  # issued together with gate_up's (MLPInLinearFn.backward)
            else:
                dw = _accumulate_weight_grad(w, dy2d, a2d)
        return dgu, dw, None


_SWIGLU_DOWN = True  # (a test seam: tests/test_model_gpu.py switches the MLP split off)


def fuse_swiglu_down() -> bool:
    """MLP split (default): gate_up GEMM | down GEMM with the SwiGLU backward fused into its dgrad. Off when the
    forward-fused gate_up + SwiGLU epilogue is requested instead (SFTAMD_TN=swiglu / 1)."""
    return _SWIGLU_DOWN and _TN_MODE not in ("1", "swiglu")


def swiglu_linear(gu: torch.Tensor, weight: torch.Tensor, box: Optional[dict] = None) -> torch.Tensor:
    """linear(swiglu(gu), weight) with the fused backward where the HIP kernels apply. box: shared with the
    mlp_in_linear that produced gu (the two weight gradients then run as one launch)."""
    if _SWIGLU_DOWN and _ext.use_hip(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous():
        return SwiGLULinearFn.apply(gu, weight, box)
    return linear(swiglu(gu), weight)


# ----------------------------------------------------------------------------- embedding
class EmbeddingFn(Function):
    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.weight = weight
        if _ext.use_hip(weight):
            return _ext.ops().embedding_fwd(ids, weight)
        return torch.nn.functional.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.weight
        if not ctx.needs_input_grad[1]:
            return None, None
        mg = getattr(w, "main_grad", None)
        flat_ids = ids.reshape(-1)
        dy2d = dy.reshape(-1, dy.shape[-1]).contiguous()
        sink = getattr(w, "_sftamd_sparse_sink", None)
        if sink is not None:
            # sparse tied-embedding gradient (DDPEngine.tied_sparse): (ids, summed rows) go to the engine, which
            # all-gathers them after backward; main_grad holds only the (early all-reduced) lm_head part. No host
            # sync: instead of torch.unique (whose output size is data-dependent) the n token rows are reduced into n
            # slots — slot s = the s-th distinct id of the sorted ids, the unused tail slots keep id 0 and a zero row
            # (an exact no-op when added)
            n = flat_ids.numel()
            sorted_ids, perm = torch.sort(flat_ids)
            head = torch.ones(n, dtype=torch.bool, device=flat_ids.device)
            if n > 1:
                head[1:] = sorted_ids[1:] != sorted_ids[:-1]
            seg = torch.cumsum(head, 0) - 1
            ids = torch.zeros(n, dtype=torch.int64, device=flat_ids.device).scatter_(0, seg, sorted_ids)
            rdt = mg.dtype if mg is not None else w.dtype
            if _ext.use_hip(dy):
                rows = torch.zeros(n, w.shape[-1], dtype=rdt, device=w.device)
                _ext.ops().embedding_bwd(dy2d, seg.to(torch.int32), perm.to(torch.int32), rows)
            else:
                rows = torch.zeros(n, w.shape[-1], dtype=torch.float32, device=w.device)
                rows.index_add_(0, seg[torch.argsort(perm)], dy2d.float())
                rows = rows.to(rdt)
            sink(ids, rows)
            return None, None
        if _ext.use_hip(dy):
            sorted_ids, perm = torch.sort(flat_ids.to(torch.int32))
            target = mg if mg is not None else torch.zeros_like(w)
            if mg is not None and getattr(w, "_sftamd_fresh", False):
                mg.zero_()  # untied embedding: the sparse row update needs a zeroed buffer
                w._sftamd_fresh = False
            _ext.ops().embedding_bwd(dy2d, sorted_ids, perm.to(torch.int32), target)
            if mg is not None:
                _weight_grad_done(w)
                return None, None
            return None, target
        g = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        g.index_add_(0, flat_ids, dy2d.float())
        return None, _accumulate_small_grad(w, g)


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    return EmbeddingFn.apply(ids, weight)


# ----------------------------------------------------------------------------- RMSNorm (+residual)
class AddRMSNormFn(Function):
    """res_out = x (+ residual); y = rmsnorm(res_out) * w. Returns (y, res_out). y_ld > H (HIP path): y is the left
    block of a [tokens, y_ld] buffer, so a LoRA-widened consumer fills its adapter columns in place (_lora_wide_prep)
    instead of copying y into its X'."""

    @staticmethod
    def forward(ctx, x, residual, weight, eps, y_ld=0):
        if _ext.use_hip(x):
            y, res_out, rstd = _ext.ops().rmsnorm_fwd(x, residual, weight, eps, int(y_ld))
        else:
            res_out = x if residual is None else (x.float() + residual.float()).to(x.dtype)
            y, rstd = ref.rms_norm(res_out, weight, eps)
        ctx.save_for_backward(res_out, rstd)
        ctx.weight = weight
        ctx.has_residual = residual is not None
        return y, res_out

    @staticmethod
    def backward(ctx, dy, dres):
        h, rstd = ctx.saved_tensors
        w = ctx.weight
        mg = getattr(w, "main_grad", None)
        if _ext.use_hip(h):
            direct = (ctx.needs_input_grad[2] and mg is not None and mg.dtype == torch.bfloat16
                      and mg.is_contiguous() and mg.data_ptr() % 8 == 0)
            # the column-sum kernel writes / accumulates dW straight into the flat gradient buffer
            dx, dw = _ext.ops().rmsnorm_bwd(dy.contiguous(), h, w, rstd,
                                           dres.contiguous() if dres is not None else None,
                                           mg if direct else None,
                                           direct and not getattr(w, "_sftamd_fresh", False))
            if direct:
                w._sftamd_fresh = False
                _weight_grad_done(w)
                return dx, (dx if ctx.has_residual else None), None, None, None
        else:
            hf = h.float()
            n = hf * rstd[..., None]
            dyf = dy.float()
            dyw = dyf * w.float()
            dx = rstd[..., None] * (dyw - n * (dyw * n).mean(-1, keepdim=True))
            if dres is not None:
                dx = dx + dres.float()
            dx = dx.to(h.dtype)
            dw = (dyf * n).reshape(-1, h.shape[-1]).sum(0)
        dweight = None
        if ctx.needs_input_grad[2]:
            dweight = _accumulate_small_grad(w, dw)
        dresid = dx if ctx.has_residual else None
        return dx, dresid, dweight, None, None


def add_rms_norm(x, residual, weight, eps, y_ld: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """(y, res_out); y_ld: see AddRMSNormFn (ignored off the HIP path). A widened y is marked with its row width
    (``_sftamd_wide_ld``): the LoRA consumer fills the rest of the row in place ONLY for a buffer marked this way,
    never for an arbitrary view whose row stride happens to match."""
    y, res = AddRMSNormFn.apply(x, residual, weight, eps, y_ld)
    if y_ld > x.shape[-1] and _ext.use_hip(x) and y.stride(-2) == y_ld:
        y._sftamd_wide_ld = int(y_ld)
    return y, res


def rms_norm(x, weight, eps) -> torch.Tensor:
    return AddRMSNormFn.apply(x, None, weight, eps)[0]


# ----------------------------------------------------------------------------- SwiGLU
class SwiGLUFn(Function):
    @staticmethod
    def forward(ctx, gate_up):
        ctx.save_for_backward(gate_up)
        if _ext.use_hip(gate_up):
            return _ext.ops().swiglu_fwd(gate_up)
        return ref.swiglu(gate_up)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        if _ext.use_hip(gu):
            return _ext.ops().swiglu_bwd(dy.contiguous(), gu)
        g, u = gu.float().chunk(2, dim=-1)
        sg = torch.sigmoid(g)
        silu = g * sg
        dyf = dy.float()
        dg = dyf * u * (sg * (1 + g * (1 - sg)))
        du = dyf * silu
        return torch.cat([dg, du], dim=-1).to(gu.dtype)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    return SwiGLUFn.apply(gate_up)


# ----------------------------------------------------------------------------- projection + fused epilogue
_TN_MODE = os.environ.get("SFTAMD_TN", "rope")  # rope | swiglu | 1 (both) | 0 (hipBLASLt + separate kernels)


def _tn_ok(x2d: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the forward-layout HIP GEMM (csrc/gemm_tn.hip, BK64 tiles of 256 x 256) handles.

    Default (measured end to end on MI355X, profiles/r1_gemm_tn.md): the qkv projection runs with the
    RoPE epilogue (beats hipBLASLt + the rope kernel); gate_up + SwiGLU stays on hipBLASLt + the SwiGLU
    kernel, because the fused kernel's GEMM core is ~5-10 % slower than hipBLASLt's on [8192, 22016] and
    that cancels the saved pass (SFTAMD_TN=1 / swiglu turns it on)."""
    return (_TN_MODE != "0" and _ext.use_hip(x2d) and x2d.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x2d.dim() == 2 and x2d.shape[0] % 256 == 0 and x2d.shape[0] > 0 and x2d.shape[1] % 64 == 0
            and x2d.stride(1) == 1 and x2d.stride(0) % 8 == 0 and w.is_contiguous() and w.shape[0] % 256 == 0)


def _tn_cfg(M: int, N: int, K: int = 64) -> int:
    """Forward GEMM with an epilogue (qkv + RoPE): the ping-pong 8-phase schedule (cfg 11, csrc/gemm_tn.hip: the two
    wave rows one barrier apart, transposed-C epilogue) wherever N % 256 == 0 — 2-6 % faster than the BK64 ring (cfg 2)
    on every SmolLM3 shape (profiles/r2_gemm_pingpong.md). The persistent row-contiguous kernel (cfg 61) is faster in
    isolation (0.121 vs 0.131 ms) but slower in the step: 137 vs 106 us per call, its 384 tiles are 1.5 rounds of one
    workgroup per CU and the cos / sin loads of its epilogue wait behind the next tile's DMA (profiles/r5_gemm_fwd.md)."""
    return 11 if N % 256 == 0 else 2


class GateUpSwiGLUFn(Function):
    """act = silu(x Wg^T) * (x Wu^T) with W = [Wg; Wu]: ONE HIP GEMM whose epilogue writes both gu (saved
    for backward) and act — the separate SwiGLU pass over the [M, 2I] output disappears."""

    @staticmethod
    def forward(ctx, x, weight):
        x2d = x.reshape(-1, x.shape[-1])
        gu, act = _ext.ops().gemm_tn_swiglu(x2d, weight, _tn_swiglu_cfg(weight))
        ctx.save_for_backward(x2d, gu)
        ctx.weight = weight
        ctx.x_shape = x.shape
        return act.view(*x.shape[:-1], act.shape[-1])

    @staticmethod
    def backward(ctx, dact):
        x2d, gu = ctx.saved_tensors
        w = ctx.weight
        dgu = _ext.ops().swiglu_bwd(dact.reshape(-1, dact.shape[-1]).contiguous(), gu)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dgu, w).view(ctx.x_shape)
        if ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dgu, x2d)
        return dx, dw


def _tn_swiglu_cfg(weight: torch.Tensor) -> int:
    """gate_up + SwiGLU epilogue (SFTAMD_TN=swiglu / 1): the persistent 4-wave kernel where it applies (0.669 vs
    0.705 ms for hipBLASLt + the SwiGLU kernel at M = 8192, profiles/r4_gemm_fwd.md), else the ping-pong kernel."""
    if weight.shape[0] % 256 == 0 and weight.shape[1] % 128 == 0:
        return _ROWC_CFG
    return 11 if weight.shape[0] % 256 == 0 else 5


def linear_swiglu(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """SwiGLU MLP input projection: swiglu(linear(x, [Wg; Wu]))."""
    x2d = x.reshape(-1, x.shape[-1])
    if _TN_MODE in ("1", "swiglu") and _tn_ok(x2d, weight) and (weight.shape[0] // 2) % 128 == 0:
        return GateUpSwiGLUFn.apply(x, weight)
    return swiglu(linear(x, weight))


class GateUpActFn(Function):
    """(gu, act) = (x [Wg; Wu]^T, silu(gate) * up) from ONE HIP GEMM with the SwiGLU epilogue; act is
    non-differentiable here because the consumer (SwiGLUDownFn) returns the gradient of gu directly."""

    @staticmethod
    def forward(ctx, x, weight):
        x2d = x.reshape(-1, x.shape[-1])
        gu, act = _ext.ops().gemm_tn_swiglu(x2d, weight, _tn_swiglu_cfg(weight))
        ctx.save_for_backward(x2d)
        ctx.weight = weight
        ctx.x_shape = x.shape
        ctx.mark_non_differentiable(act)
        # act never receives a gradient: without this autograd would zero-fill a [T, I] tensor for it every backward
        ctx.set_materialize_grads(False)
        return gu.view(*x.shape[:-1], gu.shape[-1]), act.view(*x.shape[:-1], act.shape[-1])

    @staticmethod
    def backward(ctx, dgu, _dact):
        (x2d,) = ctx.saved_tensors
        w = ctx.weight
        dgu2d = dgu.reshape(-1, dgu.shape[-1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad_mm(dgu2d, w).view(ctx.x_shape)
        if ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dgu2d, x2d)
        return dx, dw


class SwiGLUDownFn(Function):
    """y = act @ W^T for an act produced together with gu (GateUpActFn); backward = the fused
    dgu = swiglu_bwd(dy @ W, gu) GEMM of SwiGLULinearFn — neither SwiGLU pass runs as a separate kernel."""

    @staticmethod
    def forward(ctx, gu, act, weight):
        ctx.save_for_backward(gu, act)
        ctx.weight = weight
        a2d = act.reshape(-1, act.shape[-1])
        return _as_output(fwd_gemm(a2d, weight), gu.shape[:-1])

    @staticmethod
    def backward(ctx, dy):
        gu, act = ctx.saved_tensors
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1]).contiguous()
        gu2d = gu.reshape(-1, gu.shape[-1])
        dgu = dw = None
        if ctx.needs_input_grad[0]:
            if _dgrad_ok(dy2d, w):
                dgu = _ext.ops().dgrad_gemm(dy2d, w, gu2d, _dgrad_cfg(dy2d, swiglu=True))
            else:
                dgu = _ext.ops().swiglu_bwd(torch.mm(dy2d, w), gu2d)
            dgu = dgu.view(gu.shape)
        if ctx.needs_input_grad[2]:
            dw = _accumulate_weight_grad(w, dy2d, act.reshape(-1, act.shape[-1]))
        return dgu, None, dw


def swiglu_mlp(h: torch.Tensor, w_gate_up: torch.Tensor, w_down: torch.Tensor) -> torch.Tensor:
    """down(swiglu(gate_up(h))) — the SwiGLU MLP without LoRA, on the fastest available fusion:
    SFTAMD_TN=1 / swiglu: gate_up GEMM with the SwiGLU epilogue + down GEMM with the SwiGLU backward in its dgrad
    (no separate SwiGLU kernel in either direction); default: gate_up GEMM (fwd_gemm) + SwiGLU kernel + the fused
    down dgrad; otherwise the unfused chain."""
    h2d = h.reshape(-1, h.shape[-1])
    _carry_put(None)
    # (fusing it by default where gate_up has no TunableOp selection — the recipe's ragged batches — measured neutral:
    # 55.28 / 55.12 vs 55.01 / 55.04 HF, 82.84 / 82.68 vs 83.14 / 83.15 pure samples/s, r5_run22)
    fused_gu = _TN_MODE in ("1", "swiglu")
    if (fused_gu and _SWIGLU_DOWN and _tn_ok(h2d, w_gate_up) and w_gate_up.shape[0] % 256 == 0
            and (w_gate_up.shape[0] // 2) % 128 == 0):
        gu, act = GateUpActFn.apply(h, w_gate_up)
        return SwiGLUDownFn.apply(gu, act, w_down)
    if fuse_swiglu_down():
        box = {} if _WGRAD_PAIR else None
        y = swiglu_linear(mlp_in_linear(h, w_gate_up, box), w_down, box)
        _carry_put(box)  # the next layer's attention may leave its weight gradients to this MLP's launch
        return y
    return linear(linear_swiglu(h, w_gate_up), w_down)


class QKVRopeFn(Function):
    """qkv = x W^T with rotate_half RoPE applied to the q and k heads in the GEMM epilogue."""

    @staticmethod
    def forward(ctx, x, weight, cos, sin, n_q, n_kv, head_dim):
        x2d = x.reshape(-1, x.shape[-1])
        qkv = _ext.ops().gemm_tn_rope(x2d, weight, cos, sin, (n_q + n_kv) * head_dim, _tn_cfg(x2d.shape[0], weight.shape[0], x2d.shape[1]))
        ctx.save_for_backward(x2d, cos, sin)
        ctx.weight = weight
        ctx.dims = (n_q, n_kv, head_dim)
        ctx.x_shape = x.shape
        return qkv

    @staticmethod
    def backward(ctx, dqkv):
        x2d, cos, sin = ctx.saved_tensors
        w = ctx.weight
        n_q, n_kv, hd = ctx.dims
        dqkv = dqkv.contiguous()
        _rope_inplace(dqkv, cos, sin, n_q, n_kv, hd, inverse=True)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad_mm(dqkv, w).view(ctx.x_shape)
        if ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dqkv, x2d)
        return dx, dw, None, None, None, None, None


def linear_rope(x, weight, cos, sin, n_q, n_kv, head_dim):
    """rope_(linear(x, W_qkv)) on the packed [M, (n_q + 2 n_kv) * head_dim] layout."""
    x2d = x.reshape(-1, x.shape[-1])
    if (_TN_MODE in ("1", "rope") and head_dim == 128 and _tn_ok(x2d, weight) and cos.dtype == torch.float32
            and cos.is_contiguous()
            and sin.is_contiguous() and cos.shape == (x2d.shape[0], 64)):
        return QKVRopeFn.apply(x, weight, cos, sin, n_q, n_kv, head_dim)
    return rope_(linear(x, weight), cos, sin, n_q, n_kv, head_dim)


# ----------------------------------------------------------------------------- RoPE (in place on packed qkv)
class RoPEFn(Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, n_q, n_kv, head_dim):
        ctx.save_for_backward(cos, sin)
        ctx.dims = (n_q, n_kv, head_dim)
        _rope_inplace(qkv, cos, sin, n_q, n_kv, head_dim, inverse=False)
        ctx.mark_dirty(qkv)
        return qkv

    @staticmethod
    def backward(ctx, dqkv):
        cos, sin = ctx.saved_tensors
        n_q, n_kv, hd = ctx.dims
        dqkv = dqkv.contiguous()
        _rope_inplace(dqkv, cos, sin, n_q, n_kv, hd, inverse=True)
        return dqkv, None, None, None, None, None


def _rope_inplace(qkv, cos, sin, n_q, n_kv, hd, inverse):
    if _ext.use_hip(qkv):
        _ext.ops().rope_(qkv, cos, sin, n_q, n_kv, hd, inverse)
        return
    M = qkv.shape[0]
    qk = qkv[:, : (n_q + n_kv) * hd].view(M, n_q + n_kv, hd)
    qk.copy_(ref.apply_rope(qk, cos, sin, inverse=inverse))


def rope_(qkv, cos, sin, n_q, n_kv, head_dim):
    return RoPEFn.apply(qkv, cos, sin, n_q, n_kv, head_dim)


# ----------------------------------------------------------------------------- attention
class FlashAttnFn(Function):
    @staticmethod
    def forward(ctx, qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal, box=None):
        ctx.dims = (max_seqlen, n_q, n_kv, head_dim, scale, causal)
        ctx.box = box
        if _ext.use_hip(qkv):
            out, lse = _ext.ops().flash_fwd(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal)
            ctx.save_for_backward(qkv, cu_seqlens, out, lse)
            ctx.hip = True
            if box is not None and head_dim == 128:
                box["armed"] = True
        else:
            out = ref.attention(qkv, n_q, n_kv, head_dim, cu_seqlens, scale, causal)
            ctx.save_for_backward(qkv, cu_seqlens)
            ctx.hip = False
        return out

    @staticmethod
    def backward(ctx, dout):
        max_seqlen, n_q, n_kv, hd, scale, causal = ctx.dims
        if ctx.hip:
            qkv, cu, out, lse = ctx.saved_tensors
            dqkv = _ext.ops().flash_bwd(dout.contiguous(), qkv, out, lse, cu, max_seqlen, n_q, n_kv, hd, scale, causal,
                                        _take_delta(ctx.box, dout, n_q))
        else:
            qkv, cu = ctx.saved_tensors
            with torch.enable_grad():
                q = qkv.detach().float().requires_grad_(True)
                o = ref.attention(q, n_q, n_kv, hd, cu, scale, causal)
                (dq,) = torch.autograd.grad(o, q, dout.float())
            dqkv = dq.to(qkv.dtype)
        return dqkv, None, None, None, None, None, None, None, None


def flash_attention(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale=None, causal=True, delta_box=None):
    """delta_box: a fresh dict shared with attn_out_linear (the o_proj on this output): the o_proj backward computes
    the attention backward's delta in its dgrad epilogue."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    return FlashAttnFn.apply(qkv, cu_seqlens, int(max_seqlen), n_q, n_kv, head_dim, float(scale), bool(causal),
                             delta_box)


class QKVRopeAttnFn(Function):
    """attention(rope(x W_qkv^T)) as ONE autograd node: the forward is QKVRopeFn's GEMM (RoPE in the epilogue) +
    the flash forward; the backward runs flash_bwd_rope, whose dq / dK epilogues apply the inverse rotation, so the
    separate inverse-RoPE pass over dqkv (QKVRopeFn.backward) disappears. Gradients are those of
    QKVRopeFn + FlashAttnFn (tests/test_model_gpu.py)."""

    @staticmethod
    def forward(ctx, x, weight, cos, sin, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal, box=None,
                carry=None):
        ctx.box = box
        ctx.carry = carry
        if box is not None:
            box["armed"] = True
            if _WGRAD_PAIR and weight.requires_grad:  # this node's backward runs: o_proj may leave its wgrad here
                box["wgrad_pair"] = True
        x2d = x.reshape(-1, x.shape[-1])
        qkv = _ext.ops().gemm_tn_rope(x2d, weight, cos, sin, (n_q + n_kv) * head_dim,
                                      _tn_cfg(x2d.shape[0], weight.shape[0], x2d.shape[1]))
        out, lse = _ext.ops().flash_fwd(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal)
        ctx.save_for_backward(x2d, qkv, cu_seqlens, out, lse, cos, sin)
        ctx.weight = weight
        ctx.dims = (max_seqlen, n_q, n_kv, head_dim, scale, causal)
        ctx.x_shape = x.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        x2d, qkv, cu, out, lse, cos, sin = ctx.saved_tensors
        max_seqlen, n_q, n_kv, hd, scale, causal = ctx.dims
        w = ctx.weight
        dqkv = _ext.ops().flash_bwd_rope(dout.contiguous(), qkv, out, lse, cu, max_seqlen, n_q, n_kv, hd, scale, causal,
                                         cos, sin, _take_delta(ctx.box, dout, n_q))
        del qkv, out, lse
        pending = ctx.box.pop("o_wgrad", None) if ctx.box is not None else None
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = dgrad_mm(dqkv, w).view(ctx.x_shape)
        jobs = [pending] if pending is not None else []
        if ctx.needs_input_grad[1] and getattr(w, "main_grad", None) is not None:
            jobs.append((w, dqkv, x2d))
        elif ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dqkv, x2d)
        if jobs:
            _carry_or_launch(ctx.carry, jobs)
        return dx, dw, None, None, None, None, None, None, None, None, None, None, None


_ROPE_ATTN_FUSED = True  # (a test seam: tests/test_model_gpu.py compares against the two separate nodes)


def qkv_rope_attention(x, weight, cos, sin, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale=None, causal=True,
                       delta_box=None):
    """flash_attention(linear_rope(x, W_qkv, cos, sin)) — one fused autograd node when the HIP paths apply
    (the two separate nodes otherwise). delta_box: see flash_attention."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    x2d = x.reshape(-1, x.shape[-1])
    if (_ROPE_ATTN_FUSED and _TN_MODE in ("1", "rope") and head_dim == 128 and _tn_ok(x2d, weight)
            and cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()
            and cos.shape == (x2d.shape[0], 64)):
        return QKVRopeAttnFn.apply(x, weight, cos, sin, cu_seqlens, int(max_seqlen), n_q, n_kv, head_dim,
                                   float(scale), bool(causal), delta_box,
                                   _carry_take() if delta_box is not None else None)
    qkv = linear_rope(x, weight, cos, sin, n_q, n_kv, head_dim)
    return flash_attention(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal, delta_box)


# ----------------------------------------------------------------------------- LM head + CE
def _ce_rows(logits: torch.Tensor, labels: torch.Tensor, inv_count: torch.Tensor, write_grad: bool):
    """Per-row CE over the vocab. Returns stats [4, M] fp32 = (loss, lse, entropy, correct).
    If write_grad, logits is overwritten in place by d(sum(loss)*inv_count)/dlogits."""
    if _ext.use_hip(logits):
        return _ext.ops().ce_fwd(logits, labels, inv_count, write_grad)
    loss, lse, correct, ent = ref.cross_entropy(logits, labels)
    if write_grad:
        valid = (labels != IGNORE_INDEX)
        p = torch.softmax(logits.float(), -1)
        p[torch.arange(p.shape[0], device=p.device), labels.clamp(min=0)] -= 1.0
        p *= (valid.float() * inv_count.float())[:, None]
        logits.copy_(p)
    return torch.stack([loss, lse, ent, correct.float()])


class LMHeadCEFn(Function):
    """loss = sum_t CE(h_t W^T, y_t) * inv_count, with dlogits computed in the forward pass
    (written over the logits buffer), so the fp32 logits are never materialised."""

    @staticmethod
    def forward(ctx, h, weight, labels, inv_count):
        h2d = h.reshape(-1, h.shape[-1])
        logits = fwd_gemm(h2d, weight) if _ext.use_hip(h2d) else torch.nn.functional.linear(h2d, weight)
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        stats = _ce_rows(logits, labels.reshape(-1), inv_count, need_grad)
        loss = (stats[0].sum() * inv_count.float()).reshape(())
        if need_grad:
            ctx.save_for_backward(h2d, logits)
        ctx.weight = weight
        ctx.h_shape = h.shape
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, dloss, _dstats):
        h2d, dlogits = ctx.saved_tensors
        w = ctx.weight
        # the loss gradient (a device scalar: 1 for the trainer's loss.backward(), no host sync to find out) scales the
        # two [T, hidden] operands below — ~26 us per step at 16 x 512, bitwise a no-op at 1 — rather than the
        # [T, vocab] dlogits
        g = dloss.float()
        dh = dw = None
        if ctx.needs_input_grad[0]:
            dh = dgrad_mm(dlogits, w)
            if g is not None:
                dh = dh * g.to(dlogits.dtype)
            dh = dh.view(ctx.h_shape)
        if ctx.needs_input_grad[1]:
            dw = _accumulate_weight_grad(w, dlogits, h2d, scale=g)
        return dh, dw, None, None


def lm_head_cross_entropy(h, weight, labels, inv_count) -> Tuple[torch.Tensor, torch.Tensor]:
    return LMHeadCEFn.apply(h, weight, labels, inv_count)


# ----------------------------------------------------------------------------- LoRA linear
class LoRALinearFn(Function):
    """y = x W^T + scaling * concat_i(dropout(x) A_i^T B_i^T) over the sub-projections of a fused
    weight, without materialising dropout(x) twice, the per-adapter outputs, or a concatenation:
    the rank-r products are added in place into column slices of the base GEMM output."""

    @staticmethod
    def forward(ctx, x, weight, scaling, p, splits, *ab):
        n = len(ab) // 2
        As, Bs = ab[:n], ab[n:]
        x2d = x.reshape(-1, x.shape[-1])
        y = torch.nn.functional.linear(x2d, weight)
        mask = None
        xd = x2d
        if p > 0 and torch.is_grad_enabled():
            mask = torch.rand_like(x2d, dtype=torch.float32) >= p
            xd = x2d * mask.to(x2d.dtype) * (1.0 / (1.0 - p))
        xas = []
        col = 0
        for A, B, w in zip(As, Bs, splits):
            if A.numel():
                xa = torch.mm(xd, A.t())
                y[:, col:col + w].addmm_(xa, B.t(), alpha=scaling)
                xas.append(xa)
            else:
                xas.append(None)
            col += w
        ctx.save_for_backward(x2d, *(t for t in xas if t is not None), *As, *Bs)
        ctx.mask = mask
        ctx.meta = (scaling, p, tuple(splits), n, tuple(xa is not None for xa in xas), x.shape)
        ctx.weight = weight
        if x.dim() == 2:
            return y
        return y.view(*x.shape[:-1], weight.shape[0]).clone()

    @staticmethod
    def backward(ctx, dy):
        scaling, p, splits, n, has, xshape = ctx.meta
        saved = ctx.saved_tensors
        x2d = saved[0]
        k = 1 + sum(has)
        xas_it = iter(saved[1:k])
        As, Bs = saved[k:k + n], saved[k + n:k + 2 * n]
        w = ctx.weight
        dy2d = dy.reshape(-1, dy.shape[-1])
        dx = torch.mm(dy2d, w) if ctx.needs_input_grad[0] else None
        dW = None
        if ctx.needs_input_grad[1]:
            dW = _accumulate_weight_grad(w, dy2d, x2d)
        xd = x2d if ctx.mask is None else x2d * ctx.mask.to(x2d.dtype) * (1.0 / (1.0 - p))
        dAs, dBs, dxd = [], [], None
        col = 0
        for A, B, wd, h in zip(As, Bs, splits, has):
            if not h:
                dAs.append(None)
                dBs.append(None)
                col += wd
                continue
            xa = next(xas_it)
            dyi = dy2d[:, col:col + wd]
            dBs.append(torch.mm(dyi.t(), xa).mul_(scaling).to(B.dtype))
            t = torch.mm(dyi, B)
            dAs.append(torch.mm(t.t(), xd).mul_(scaling).to(A.dtype))
            c = torch.mm(t, A).mul_(scaling)
            dxd = c if dxd is None else dxd.add_(c)
            col += wd
        if dx is not None and dxd is not None:
            if ctx.mask is not None:
                dxd = dxd * ctx.mask.to(dxd.dtype) * (1.0 / (1.0 - p))
            dx = dx + dxd
        if dx is not None:
            dx = dx.view(xshape)
        return (dx, dW, None, None, None, *dAs, *dBs)


def dropout_add(a: Optional[torch.Tensor], b: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """(a or 0) + dropout(b) with a counter-hash mask (regenerable from seed; see csrc/elementwise.hip)."""
    if _ext.use_hip(b):
        return _ext.ops().dropout_add(a, b, float(p), int(seed))
    return ref.dropout_add(a, b, p, seed)


def lora_inplace_ok(K: int, R: int) -> bool:
    """Shapes csrc/lora.hip's widening kernels (lora_fwd / lora_fwd_inplace) take: K % 256, R = r x active
    sub-projections a multiple of 16 in [16, 64]."""
    return K % 256 == 0 and R % 16 == 0 and 16 <= R <= 64


def _lora_hip(x2d, acat) -> bool:
    return _ext.use_hip(x2d) and lora_inplace_ok(x2d.shape[1], acat.shape[0])


def _lora_fwd(x2d, acat, s, p, seed, ldX=0, swiglu=False):
    """X' = [x | s dropout(x) A^T | 0]; dropout(x) is not saved (lora_tsum regenerates the mask from the seed). swiglu:
    x2d is gu [T, 2K] and x = silu(gate) * up is formed on the fly (no SwiGLU pass, no act tensor)."""
    if _lora_hip(x2d, acat):
        return _ext.ops().lora_fwd(x2d, acat, float(s), float(p), int(seed), int(ldX), False, bool(swiglu))[0]
    if swiglu:
        x2d = ref.swiglu(x2d.float()).to(x2d.dtype)
    return ref.lora_fwd(x2d, acat, s, p, seed, ldX)[0]


def _lora_tsum(Xm, K, S, p, seed) -> torch.Tensor:
    """S^T dropout(Xm[:, :K]) in fp32 (the forward's mask regenerated from the seed when p > 0): one pass over the
    wide operand (csrc/lora.hip tsum_kernel), returned as [splits, R, K] partial sums over token chunks on the HIP
    path (summed by lora_grad_out as it scatters them, or by _scatter_grads' fallback), [R, K] otherwise."""
    R = S.shape[1]
    if (_ext.use_hip(Xm) and Xm.dtype == torch.bfloat16 and S.dtype == torch.bfloat16 and K % 8 == 0
            and R % 16 == 0 and 16 <= R <= 64 and Xm.stride(1) == 1 and Xm.stride(0) % 8 == 0 and S.stride(1) == 1
            and S.stride(0) % 8 == 0 and S.data_ptr() % 16 == 0):
        return _ext.ops().lora_tsum(Xm, int(K), S, float(p), int(seed))
    xs = ref.dropout_add(None, Xm[:, :K], p, seed) if p > 0 else Xm[:, :K]
    return S.float().t() @ xs.float()


def _scatter_direct(total: torch.Tensor, params):
    """The main_grad slices ``params``' gradients go to when lora_grad_out can write them directly, else None."""
    mgs = [getattr(p, "main_grad", None) for p in params]
    if (all(m is not None for m in mgs) and _ext.use_hip(total) and len(params) <= 4
            and all(m.is_contiguous() and m.dtype in (torch.bfloat16, torch.float32) for m in mgs)):
        return mgs
    return None


def _scatter_done(params):
    for p in params:
        p._sftamd_fresh = False
        _weight_grad_done(p)
    return [None] * len(params)


def _scatter_pair(tot_b, Bs, blocks_b, tot_a, As, blocks_a):
    """A projection's dB^T and dA scatters (_scatter_grads) in ONE lora_grad_out2 launch when both go straight into
    main_grad."""
    mb, ma = _scatter_direct(tot_b, Bs), _scatter_direct(tot_a, As)
    if mb is None or ma is None:
        return _scatter_grads(tot_b, Bs, blocks_b, tr=True), _scatter_grads(tot_a, As, blocks_a, tr=False)
    acc = [[0 if getattr(p, "_sftamd_fresh", False) else 1 for p in ps] for ps in (Bs, As)]
    _ext.ops().lora_grad_out2(tot_b, mb, [b[0] for b in blocks_b], [b[1] for b in blocks_b], True, acc[0],
                              tot_a, ma, [b[0] for b in blocks_a], [b[1] for b in blocks_a], False, acc[1])
    return _scatter_done(Bs), _scatter_done(As)


def _scatter_grads(total: torch.Tensor, params, blocks, tr: bool):
    """Per-adapter gradients from one fp32 sum [R, K]: param q's block starts at (r0, c0) of ``total`` (transposed when
    ``tr``). With DDP main_grad slices they are written / accumulated in ONE launch and None is returned to autograd;
    otherwise the blocks are returned."""
    shapes = [(p.shape[1], p.shape[0]) if tr else tuple(p.shape) for p in params]
    mgs = _scatter_direct(total, params)
    if mgs is not None:
        acc = [0 if getattr(p, "_sftamd_fresh", False) else 1 for p in params]
        _ext.ops().lora_grad_out(total, mgs, [b[0] for b in blocks], [b[1] for b in blocks], bool(tr), acc)
        return _scatter_done(params)
    if total.dim() == 3:
        total = total.sum(0)
    out = []
    for p, (r0, c0), (nr, nc) in zip(params, blocks, shapes):
        g = total[r0:r0 + nr, c0:c0 + nc]
        out.append(_accumulate_small_grad(p, g.t() if tr else g))
    return out


def _lora_dxa(dy2d: torch.Tensor, bc: torch.Tensor, s: float, meta=None, r: int = 0) -> torch.Tensor:
    """s dy Bc for the adapters' B columns Bc [n, R] of the wide weight (a thin-N GEMM: the HIP streaming kernels where
    the layout allows, torch.addmm with the scale as alpha otherwise). ``meta`` [(o, rows, c)] / ``r``: Bc's
    block-diagonal layout (sub-projection rows [o, o + rows) x columns [c, c + r), zero elsewhere)."""
    R = bc.shape[1]
    if not (_ext.use_hip(dy2d) and dy2d.dtype == torch.bfloat16 and bc.dtype == torch.bfloat16 and R % 16 == 0
            and 16 <= R <= 64 and dy2d.stride(1) == 1 and dy2d.stride(0) % 8 == 0 and dy2d.data_ptr() % 16 == 0
            and dy2d.shape[1] % 8 == 0 and bc.stride(1) == 1 and bc.stride(0) % 8 == 0 and bc.data_ptr() % 16 == 0):
        return torch.addmm(dy2d.new_empty(dy2d.shape[0], R), dy2d, bc, beta=0, alpha=s)
    # several sub-projections (qkv, gate_up): the block kernel reads each block's dy columns against only that block's
    # r columns, in pieces (gate_up 89.5 vs 107.0 us for addmm and 135.1 for the dense kernel, which re-reads all of
    # Bc per 32 token rows; qkv 17.8 vs 23.9 dense; r5_run20); one block (o, down): the dense kernel (13.0-13.2 vs 14.4)
    if (meta is not None and len(meta) > 1 and r in (16, 32) and len(meta) <= 4
            and all(o % 8 == 0 and c % 8 == 0 for o, _, c in meta)):
        return _ext.ops().lora_dxa_blocks(dy2d, bc, [m[0] for m in meta], [m[1] for m in meta], [m[2] for m in meta],
                                          int(r), float(s))
    if dy2d.shape[1] <= 4096:
        return _ext.ops().lora_dxa(dy2d, bc, float(s))
    return torch.addmm(dy2d.new_empty(dy2d.shape[0], R), dy2d, bc, beta=0, alpha=s)


def _lora_bwd_dx(base, dxa, acat, p, seed, gu=None):
    """dx = base + dropout(dxa A_cat); with gu (the SwiGLU input of a LoRA MLP's down projection) dgu =
    swiglu_bwd(dx, gu) instead, in the same pass (csrc/lora.hip bwd_dx_kernel: no dx round trip)."""
    if _ext.use_hip(base) and acat.shape[0] % 16 == 0 and acat.shape[0] <= 64:
        return _ext.ops().lora_bwd_dx(base, dxa, acat, float(p), int(seed), gu)
    dx = ref.lora_bwd_dx(base, dxa, acat, p, seed)
    return dx if gu is None else swiglu_bwd(dx, gu)


_PARAM_EPOCH = [0]


def bump_param_epoch() -> None:
    """Called by the optimizers after every update they issue (parameters change in place through a raw-pointer
    kernel, which no tensor's version counter sees)."""
    _PARAM_EPOCH[0] += 1


_PARAM_SYNCS: list = []  # weak refs to the overlapped optimizers' synchronize(): order the stream after the updates


def register_param_sync(fn) -> None:
    """An optimizer that runs its update on a side stream under the next forward registers its ``synchronize`` here.
    A copy that reads MANY layers' parameters at once (the batched LoRA wide-weight refresh) calls every registered
    one first: the per-layer forward pre-hooks only order each layer after its OWN update / all-gather."""
    _PARAM_SYNCS[:] = [r for r in _PARAM_SYNCS if r() is not None and r() != fn]
    _PARAM_SYNCS.append(weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda f=fn: f))


def _await_param_updates() -> None:
    for r in list(_PARAM_SYNCS):
        f = r()
        if f is not None:
            f()


def _sync_wide(wide: torch.Tensor, K: int, r: int, meta, Bs) -> None:
    """Copy the adapters' B matrices into their blocks of the wide weight — only when one may have changed since
    the last copy: an optimizer update (the parameter epoch) or an in-place edit / checkpoint load (the Bs' version
    counters). GA micro-batches and eval passes between two updates copy nothing."""
    key = (_PARAM_EPOCH[0],) + tuple((B._version, B.data_ptr()) for B in Bs)
    if getattr(wide, "_sftamd_bkey", None) == key:
        return
    _await_param_updates()
    with torch.no_grad():
        for (o, rows, c), B in zip(meta, Bs):
            wide[o:o + rows, K + c:K + c + r].copy_(B)
    wide._sftamd_bkey = key


class _WideEntry:
    """A wide weight's adapters on the HIP path: the B blocks it holds, its persistent A_cat buffer, the key of the
    parameter state they were last copied from, and their copy descriptors."""
    __slots__ = ("ids", "K", "r", "meta", "As", "Bs", "acat", "key")

    def __init__(self, wide, K, r, meta, As, Bs):
        self.ids = tuple(id(t) for t in (*As, *Bs))
        self.K, self.r, self.meta, self.As, self.Bs = K, r, tuple(meta), list(As), list(Bs)
        self.acat = torch.empty(r * len(As), K, device=wide.device, dtype=wide.dtype)
        self.key = None

    def state(self):
        return (_PARAM_EPOCH[0],) + tuple((t._version, t.data_ptr()) for t in (*self.As, *self.Bs))

    def descs(self, wide):
        ld, K, r, es = wide.stride(0), self.K, self.r, wide.element_size()
        d = [(B.data_ptr(), wide.data_ptr() + es * (o * ld + K + c), rows, r, B.stride(0), ld)
             for (o, rows, c), B in zip(self.meta, self.Bs)]
        d += [(A.data_ptr(), self.acat.data_ptr() + es * i * r * K, r, K, A.stride(0), K) for i, A in enumerate(self.As)]
        return d


_WIDE_REG: list = []        # weakrefs to the wide weights on the HIP path
_WIDE_TABLE = [None, None]  # (descriptor-set key, (device table, max elements)) of the last batched sync


def _wide_sync(wide, K, r, meta, As, Bs) -> torch.Tensor:
    """The HIP path's _sync_wide + A concatenation: returns this projection's persistent A_cat. When any adapter may
    have changed (the same epoch / version keys as _sync_wide), EVERY registered wide weight that is stale — after an
    optimizer step, all of them — is refreshed by one copy2d_batch launch (B blocks into W', A rows into A_cat); the
    device descriptor table is rebuilt only when the set of copies or their addresses change."""
    ent = getattr(wide, "_sftamd_sync", None)
    if ent is None or ent.ids != tuple(id(t) for t in (*As, *Bs)):
        ent = _WideEntry(wide, K, r, meta, As, Bs)
        wide._sftamd_sync = ent
        _WIDE_REG.append(weakref.ref(wide))
    if ent.key == ent.state():
        return ent.acat
    live = [w for w in (ref() for ref in _WIDE_REG) if w is not None]
    _WIDE_REG[:] = [weakref.ref(w) for w in live]
    stale = [w for w in live if w.device == wide.device and w._sftamd_sync.key != w._sftamd_sync.state()]
    rows = [d for w in stale for d in w._sftamd_sync.descs(w)]
    tkey = tuple(rows)
    if _WIDE_TABLE[0] != tkey:
        table = torch.tensor(rows, dtype=torch.int64).to(wide.device)
        _WIDE_TABLE[0], _WIDE_TABLE[1] = tkey, (table, max(d[2] * d[3] for d in rows))
    table, most = _WIDE_TABLE[1]
    # the copy reads every stale layer's adapters: wait for ALL overlapped updates / ZeRO-1 gathers first (LoRA's
    # update is a few MB, so the overlap it gives up is negligible)
    _await_param_updates()
    _ext.ops().copy2d_batch(table, int(most))
    for w in stale:
        w._sftamd_sync.key = w._sftamd_sync.state()
    return ent.acat


def _wide_sync_ok(wide, As, Bs) -> bool:
    return (_ext.use_hip(wide) and wide.dtype == torch.bfloat16 and wide.stride(1) == 1
            and all(t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.device == wide.device for t in (*As, *Bs)))


def _lora_gemm(X: torch.Tensor, wide: torch.Tensor) -> torch.Tensor:
    """The widened LoRA forward GEMM X' W'^T: the routing rule of fwd_gemm (hipBLASLt where TunableOp holds a selection
    for the exact wide shape, SFTAMD_FWD_GEMM), else the hand-written persistent kernel with the row-contiguous store
    epilogue (113.0 samples/s vs 112.9 for untuned hipBLASLt, profiles/r4_lora.md; profiles/r5_gemm_fwd.md)."""
    if _fwd_on_hip(X, wide) and X.is_contiguous():
        return _ext.ops().gemm_tn(X, wide, _LORA_FWD_CFG)
    return torch.mm(X, wide.t())


# the persistent 4-wave kernel with the row-contiguous nt store epilogue (csrc/gemm_tn.hip cfg 61): 131.3 vs 130.2
# samples/s for cfg 164 (r5_run08, one box)
_LORA_FWD_CFG = int(os.environ.get("SFTAMD_LORA_FWD_CFG", "61"))


def _lora_wide_prep(x, wide, K, scaling, p, seed, meta, ab, swiglu=False):
    """X' = [x | s dropout(x) A_cat^T | 0] for the wide GEMM (and the adapters' B blocks synced into W'); swiglu: x is
    the SwiGLU input gu [.., 2K] and the activation silu(gate) * up is formed inside lora_fwd."""
    n = len(ab) // 2
    As, Bs = ab[:n], ab[n:]
    r = As[0].shape[0]
    x2d = x.reshape(-1, 2 * K if swiglu else K)
    if _wide_sync_ok(wide, As, Bs):
        acat = _wide_sync(wide, K, r, meta, As, Bs)
    else:
        _sync_wide(wide, K, r, meta, Bs)
        acat = As[0].contiguous() if n == 1 else torch.cat(As, 0)
    X = _prewidened(x, x2d, wide.shape[1], acat) if not swiglu else None
    if X is not None:  # x was written into X's left block by its producer (add_rms_norm y_ld): fill the rest in place
        _ext.ops().lora_fwd_inplace(X, K, acat, float(scaling), float(p), int(seed))
    else:
        X = _lora_fwd(x2d.contiguous(), acat, scaling, p, seed, wide.shape[1], swiglu)
    return X, acat, (K, r * n, r, n, float(scaling), float(p), int(seed), tuple(meta), x.shape)


def _prewidened(x: torch.Tensor, x2d: torch.Tensor, ldX: int, acat: torch.Tensor) -> Optional[torch.Tensor]:
    """X [T, ldX] when x is a norm output add_rms_norm wrote as the left block of its own [T, ldX] buffer (marked
    ``_sftamd_wide_ld``) and the in-place widening kernel takes the shape; else None (the copying path)."""
    T, K = x2d.shape
    if (getattr(x, "_sftamd_wide_ld", 0) != ldX or not _lora_hip(x2d, acat)
            or T == 0 or K >= ldX or x2d.stride(1) != 1 or x2d.stride(0) != ldX
            or x2d.dtype != torch.bfloat16 or x2d.data_ptr() % 16 != 0):
        return None
    st = x2d.untyped_storage()
    if (x2d.storage_offset() + T * ldX) * x2d.element_size() > st.nbytes():
        return None
    return x2d.as_strided((T, ldX), (ldX, 1))


def _lora_wide_bwd(X, acat, wide, ab, state, dy2d, need_dx, gu=None):
    """The wide LoRA backward (see LoRAWideFn). Returns (dx — or dgu = swiglu_bwd(dx, gu) when gu is given —, dAs,
    dBs); the adapter gradients are None where they went straight into main_grad."""
    K, R, r, n, scaling, p, seed, meta, _ = state
    As, Bs = ab[:n], ab[n:]
    if not dy2d.is_contiguous():
        dy2d = dy2d.contiguous()
    base = dgrad_mm(dy2d, wide[:, :K])              # [T, K] (HIP 4-wave dgrad where the shapes allow)
    # dxa = s dy B_blockdiag [T, R]: one streaming pass over dy (csrc/lora.hip dxa_kernel, the scale in its epilogue)
    dxa = _lora_dxa(dy2d, wide[:, K:K + R], scaling, meta, r)
    # the adapter gradients of all sub-projections, each from one pass over its wide operand, scattered straight into
    # the parameters' flat gradient slices in one launch (no per-adapter GEMMs, slicing copies or autograd
    # accumulation): dB^T = (s xa)^T dy [R, n_out] (block (c_i, o_i) transposed is dB_i); dA = dxa^T dropout(x)
    # [R, K] (the forward's dropout mask regenerated from the seed: nothing saved)
    n_out = dy2d.shape[1]
    dBs, dAs = _scatter_pair(_lora_tsum(dy2d, n_out, X[:, K:K + R], 0.0, 0), Bs, [(c, o) for (o, rows, c) in meta],
                             _lora_tsum(X, K, dxa, p, seed), As, [(i * r, 0) for i in range(n)])
    dx = _lora_bwd_dx(base, dxa, acat, p, seed, gu) if need_dx else None
    return dx, dAs, dBs


def swiglu_bwd(dact: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    """dgu = d(silu(gate) * up) / d(gate, up) for the upstream dact (the SwiGLU kernel's backward)."""
    if _ext.use_hip(gu):
        return _ext.ops().swiglu_bwd(dact.contiguous(), gu)
    g, u = gu.float().chunk(2, dim=-1)
    sg = torch.sigmoid(g)
    d = dact.float()
    return torch.cat([d * u * (sg * (1 + g * (1 - sg))), d * g * sg], dim=-1).to(gu.dtype)


class LoRAWideFn(Function):
    """LoRA folded into the base GEMM (models.lora.FusedLoRA.wide).

    The frozen base weight W [n, K] lives in the left columns of W' = [W | B_blockdiag | 0] [n, K+Rp]
    (R = r x active sub-projections, padded to Rp = a multiple of 128); the activation is widened the same way,
    X' = [x | s * xa | 0] with xa = dropout(x) A_cat^T (csrc/lora.hip lora_fwd: one pass over x). Then
        forward:  y = X' W'^T                      (one HIP GEMM, K+Rp deep: no rank-r pass over y)
        backward: base = dy W                      (the 4-wave HIP dgrad on W's column block of W')
                  dxa  = s dy B_blockdiag          (thin [T, R] product, s as the GEMM's alpha)
                  dB^T = (s xa)^T dy, dA = dxa^T dropout(x) (csrc/lora.hip tsum: one pass over dy / x each, the
                                                   dropout mask regenerated from the seed; scattered into main_grad)
                  dx = base + dropout(dxa A_cat)   (csrc/lora.hip lora_bwd_dx: one pass)"""

    @staticmethod
    def forward(ctx, x, wide, K, scaling, p, seed, meta, *ab):
        X, acat, state = _lora_wide_prep(x, wide, K, scaling, p, seed, meta, ab)
        y = _lora_gemm(X, wide)
        ctx.save_for_backward(X, acat)
        ctx.wide, ctx.adapters, ctx.meta = wide, ab, state  # adapter gradients go to main_grad directly
        if x.dim() == 2:
            return y
        return y.view(*x.shape[:-1], wide.shape[0])

    @staticmethod
    def backward(ctx, dy):
        X, acat = ctx.saved_tensors
        dx, dAs, dBs = _lora_wide_bwd(X, acat, ctx.wide, ctx.adapters, ctx.meta, dy.reshape(-1, dy.shape[-1]),
                                      ctx.needs_input_grad[0])
        if dx is not None:
            dx = dx.view(ctx.meta[-1])
        return (dx, None, None, None, None, None, None, *dAs, *dBs)


class LoRAGateUpFn(Function):
    """gu = the LoRA-widened gate_up GEMM (its SwiGLU is formed by the consumer, LoRASwiGLUDownFn, inside the down
    projection's widening pass). (The persistent GEMM's SwiGLU epilogue writing gu and act measured slower than the
    plain wide GEMM + the SwiGLU kernel: 688 vs ~665 us at 8192 x 22016, r4_run20.)"""

    @staticmethod
    def forward(ctx, x, wide, K, scaling, p, seed, meta, *ab):
        X, acat, state = _lora_wide_prep(x, wide, K, scaling, p, seed, meta, ab)
        gu = _lora_gemm(X, wide)
        ctx.save_for_backward(X, acat)
        ctx.wide, ctx.adapters, ctx.meta = wide, ab, state
        return gu.view(*x.shape[:-1], gu.shape[-1])

    @staticmethod
    def backward(ctx, dgu):
        X, acat = ctx.saved_tensors
        dx, dAs, dBs = _lora_wide_bwd(X, acat, ctx.wide, ctx.adapters, ctx.meta, dgu.reshape(-1, dgu.shape[-1]),
                                      ctx.needs_input_grad[0])
        if dx is not None:
            dx = dx.view(ctx.meta[-1])
        return (dx, None, None, None, None, None, None, *dAs, *dBs)


class LoRASwiGLUDownFn(Function):
    """y = the LoRA-widened down projection of silu(gate) * up: the widening pass reads gu and forms the activation on
    the fly (csrc/lora.hip lora_fwd swiglu: no SwiGLU kernel, no act tensor); the backward applies the SwiGLU backward
    inside the adapter-dx pass and returns dgu (the gradient of gu) directly."""

    @staticmethod
    def forward(ctx, gu, wide, K, scaling, p, seed, meta, *ab):
        X, acat, state = _lora_wide_prep(gu, wide, K, scaling, p, seed, meta, ab, swiglu=True)
        y = _lora_gemm(X, wide)
        ctx.save_for_backward(X, acat, gu)
        ctx.wide, ctx.adapters, ctx.meta = wide, ab, state
        return y.view(*gu.shape[:-1], wide.shape[0])

    @staticmethod
    def backward(ctx, dy):
        X, acat, gu = ctx.saved_tensors
        gu2d = gu.reshape(-1, gu.shape[-1])
        dgu, dAs, dBs = _lora_wide_bwd(X, acat, ctx.wide, ctx.adapters, ctx.meta, dy.reshape(-1, dy.shape[-1]),
                                       ctx.needs_input_grad[0], gu=gu2d)
        if dgu is not None:
            dgu = dgu.view(gu.shape)
        return (dgu, None, None, None, None, None, None, *dAs, *dBs)


def _lora_wide_args(lora, weight):
    """(wide args, As, Bs) when the adapter runs on the wide path for this weight, else None."""
    wide = getattr(lora, "wide", None)
    if wide is None or weight.data_ptr() != wide.data_ptr() or weight.shape[1] != lora.in_features:
        return None
    As = [a for a, act in zip(lora.A, lora.active) if act]
    Bs = [b for b, act in zip(lora.B, lora.active) if act]
    if not As:
        return None
    p = lora.dropout.p if isinstance(lora.dropout, torch.nn.Dropout) and lora.training else 0.0
    seed = int(torch.randint(1, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
    return (wide, lora.in_features, float(lora.scaling), float(p), seed, tuple(lora.wide_meta)), As, Bs


def lora_swiglu_mlp(h, w_gate_up, w_down, l_gate_up, l_down) -> torch.Tensor:
    """down(swiglu(gate_up(h))) with LoRA adapters on both projections: on the HIP wide path one node per projection,
    the SwiGLU formed inside the down projection's widening pass and its backward inside the adapter-dx pass (the
    node returns dgu); otherwise the plain composition of lora_linear and swiglu."""
    _carry_put(None)
    gu_args, dn_args = _lora_wide_args(l_gate_up, w_gate_up), _lora_wide_args(l_down, w_down)
    h2d = h.reshape(-1, h.shape[-1])
    if (gu_args is not None and dn_args is not None and _ext.use_hip(h2d) and h2d.shape[0] % 256 == 0
            and gu_args[0][0].shape[0] % 256 == 0 and (gu_args[0][0].shape[0] // 2) % 128 == 0
            and gu_args[0][0].shape[1] % 128 == 0):
        (a, ga_As, ga_Bs), (b, dn_As, dn_Bs) = gu_args, dn_args
        gu = LoRAGateUpFn.apply(h, *a, *ga_As, *ga_Bs)
        return LoRASwiGLUDownFn.apply(gu, *b, *dn_As, *dn_Bs)
    return lora_linear(swiglu(lora_linear(h, w_gate_up, l_gate_up)), w_down, l_down)


class LoRAQKVRopeAttnFn(Function):
    """attention(rope(x' W'^T)) for a LoRA-adapted qkv projection as ONE autograd node (the LoRA twin of
    QKVRopeAttnFn): the widened activation X' (lora_fwd) goes through the forward GEMM with the RoPE epilogue, the
    backward's flash_bwd_rope applies the inverse rotation in its dq / dK epilogues, and its dqkv feeds the wide LoRA
    backward (base dgrad, adapter dx, dA / dB straight into main_grad) — no separate RoPE pass either way."""

    @staticmethod
    def forward(ctx, x, cos, sin, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal, wide, K, scaling, p,
                seed, meta, *ab):
        X, acat, state = _lora_wide_prep(x, wide, K, scaling, p, seed, meta, ab)
        qkv = _ext.ops().gemm_tn_rope(X, wide, cos, sin, (n_q + n_kv) * head_dim, _tn_cfg(X.shape[0], wide.shape[0], X.shape[1]))
        out, lse = _ext.ops().flash_fwd(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal)
        ctx.save_for_backward(X, acat, qkv, cu_seqlens, out, lse, cos, sin)
        ctx.wide, ctx.adapters, ctx.meta = wide, ab, state
        ctx.dims = (max_seqlen, n_q, n_kv, head_dim, scale, causal)
        return out

    @staticmethod
    def backward(ctx, dout):
        X, acat, qkv, cu, out, lse, cos, sin = ctx.saved_tensors
        max_seqlen, n_q, n_kv, hd, scale, causal = ctx.dims
        dqkv = _ext.ops().flash_bwd_rope(dout.contiguous(), qkv, out, lse, cu, max_seqlen, n_q, n_kv, hd, scale, causal,
                                         cos, sin)
        del qkv, out, lse
        dx, dAs, dBs = _lora_wide_bwd(X, acat, ctx.wide, ctx.adapters, ctx.meta, dqkv, ctx.needs_input_grad[0])
        if dx is not None:
            dx = dx.view(ctx.meta[-1])
        return (dx, None, None, None, None, None, None, None, None, None, None, None, None, None, None, None,
                *dAs, *dBs)


def lora_qkv_rope_attention(x, weight, lora, cos, sin, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale=None,
                            causal=True):
    """flash_attention(rope_(lora_linear(x, W_qkv, lora))) — one fused autograd node on the HIP wide path
    (LoRAQKVRopeAttnFn), the composition of the three otherwise."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    args = _lora_wide_args(lora, weight)
    x2d = x.reshape(-1, x.shape[-1])
    if (args is not None and _ROPE_ATTN_FUSED and head_dim == 128 and _ext.use_hip(x2d)
            and x2d.shape[0] % 256 == 0 and args[0][0].shape[0] % 256 == 0 and args[0][0].shape[1] % 128 == 0
            and cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()
            and cos.shape == (x2d.shape[0], 64)):
        a, As, Bs = args
        return LoRAQKVRopeAttnFn.apply(x, cos, sin, cu_seqlens, int(max_seqlen), n_q, n_kv, head_dim, float(scale),
                                       bool(causal), *a, *As, *Bs)
    qkv = rope_(lora_linear(x, weight, lora), cos, sin, n_q, n_kv, head_dim)
    return flash_attention(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, causal)


def lora_linear(x, weight, lora) -> torch.Tensor:
    """``lora``: a models.lora.FusedLoRA module (adapters per sub-projection)."""
    w = _lora_wide_args(lora, weight)
    if w is not None:
        a, As, Bs = w
        return LoRAWideFn.apply(x, *a, *As, *Bs)
    p = lora.dropout.p if isinstance(lora.dropout, torch.nn.Dropout) and lora.training else 0.0
    return LoRALinearFn.apply(x, weight, float(lora.scaling), float(p), tuple(lora.out_splits), *lora.A, *lora.B)


def decode_attention(q, kcache, vcache, cache_len, n_q, n_kv, scale=None):
    """Single-token GQA attention over cache[:cache_len] (cache_len: int32 device tensor)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.numel() // n_q)
    if _ext.use_hip(q):
        return _ext.ops().decode_attention(q, kcache, vcache, cache_len, n_q, n_kv, float(scale))
    L = int(cache_len.item())
    D = q.numel() // n_q
    qg = q.float().view(n_kv, n_q // n_kv, D)
    att = torch.einsum("grd,sgd->grs", qg, kcache[:L].float()) * scale
    return torch.einsum("grs,sgd->grd", att.softmax(-1), vcache[:L].float()).reshape(-1).to(q.dtype)
