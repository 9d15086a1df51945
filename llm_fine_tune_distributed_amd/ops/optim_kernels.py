"""Flat-buffer optimizer kernels: global grad-norm + fused AdamW.

The DDP engine keeps every trainable parameter, its gradient, the fp32 master copy and
the Adam moments in a handful of large contiguous buffers, so one kernel launch updates
the whole model at HBM bandwidth (no multi-tensor pointer lists). The clip coefficient
stays on the device (no host sync between the norm and the update).
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch

from . import _ext
from . import reference as ref


def sumsq_list(tensors) -> torch.Tensor:
    """fp32 sum of squares over a list of (bf16) tensors: one HIP partial-sum kernel per tensor, one
    concatenated reduction (ZeRO-1 grad norm over the owned gradient slices)."""
    tensors = [t for t in tensors if t.numel() > 0]
    if not tensors:
        return torch.zeros((), dtype=torch.float32)
    if _ext.use_hip(tensors[0]):
        return torch.cat([_ext.ops().sumsq(t) for t in tensors]).sum()
    return sum(t.float().pow(2).sum() for t in tensors)


def grad_norm_flat(grads: Iterable[torch.Tensor], max_norm: float):
    """Returns (total_norm, clip_coef) as fp32 [1] tensors on the grads' device."""
    grads = [g for g in grads if g.numel() > 0]
    dev = grads[0].device
    total = torch.zeros(1, dtype=torch.float32, device=dev)
    for g in grads:
        if _ext.use_hip(g):
            total += _ext.ops().sumsq(g).sum()
        else:
            total += g.float().pow(2).sum()
    norm = total.sqrt()
    if max_norm is None or max_norm <= 0:
        coef = torch.ones_like(norm)
    else:
        coef = (max_norm / (norm + 1e-6)).clamp(max=1.0)
    return norm, coef


def adamw_flat_(param: torch.Tensor, grad: torch.Tensor, master: Optional[torch.Tensor],
                exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, clip_coef: torch.Tensor,
                lr: float, beta1: float, beta2: float, eps: float, weight_decay: float, step: int,
                sr_seed: int = 0, sr_offset: int = 0) -> None:
    """In-place AdamW on flat buffers. grad is multiplied by clip_coef (device scalar).
    Moments are fp32 or bf16 (both the same). Without a master copy, ``sr_seed != 0`` writes the
    bf16 parameters (and bf16 moments) with stochastic rounding."""
    if param.numel() == 0:
        return
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if _ext.use_hip(param):
        _ext.ops().adamw_flat(param, grad, master, exp_avg, exp_avg_sq, clip_coef,
                              float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                              float(bc1), float(bc2), int(sr_seed), int(sr_offset))
        return
    g = grad.float() * clip_coef.float()
    ref.adamw_(param, g, exp_avg, exp_avg_sq, master, lr, beta1, beta2, eps, weight_decay, step,
               sr_seed=sr_seed, sr_offset=sr_offset)
