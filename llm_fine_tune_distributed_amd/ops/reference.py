"""Pure-PyTorch reference implementations of every fused op.

These run on CPU (tests, the gloo plumbing config of BASELINE.json) and serve as the fp32
numerics oracle for the HIP kernels. Semantics follow the HF modules the reference runs
(transformers ``modeling_smollm3.py``: RMSNorm, rotate_half RoPE, SwiGLU, causal GQA SDPA,
``loss_utils.py`` ForCausalLMLoss with ignore_index=-100 and sum/num_items normalisation).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

IGNORE_INDEX = -100


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (y, rstd). y = weight * x / sqrt(mean(x^2) + eps), computed in fp32."""
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    y = (xf * rstd).to(x.dtype) * weight
    return y, rstd.squeeze(-1)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    g, u = gate_up.chunk(2, dim=-1)
    return (F.silu(g.float()) * u.float()).to(gate_up.dtype)


def rope_cos_sin(positions: torch.Tensor, head_dim: int, theta: float,
                 scaling: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """cos/sin tables [n, head_dim/2] in fp32 for the given integer positions."""
    inv_freq = rope_inv_freq(head_dim, theta, scaling, positions.device)
    freqs = positions.float()[:, None] * inv_freq[None, :]
    return freqs.cos(), freqs.sin()


def rope_inv_freq(head_dim: int, theta: float, scaling: Optional[dict], device=None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64, device=device) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(is_mid, mid, scaled)
    return inv.float()


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, inverse: bool = False) -> torch.Tensor:
    """x [M, H, D]; cos/sin [M, D/2]. rotate_half convention (HF Llama/SmolLM3)."""
    d2 = x.shape[-1] // 2
    xf = x.float()
    x1, x2 = xf[..., :d2], xf[..., d2:]
    c, s = cos[:, None, :], sin[:, None, :]
    if inverse:
        s = -s
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    return torch.cat([o1, o2], dim=-1).to(x.dtype)


def attention(qkv: torch.Tensor, n_q: int, n_kv: int, head_dim: int, cu_seqlens: torch.Tensor,
              scale: Optional[float] = None, causal: bool = True) -> torch.Tensor:
    """Varlen causal GQA attention on the packed qkv layout [M, (n_q+2n_kv)*D] -> [M, n_q*D]."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    M = qkv.shape[0]
    q = qkv[:, : n_q * head_dim].view(M, n_q, head_dim)
    k = qkv[:, n_q * head_dim: (n_q + n_kv) * head_dim].view(M, n_kv, head_dim)
    v = qkv[:, (n_q + n_kv) * head_dim:].view(M, n_kv, head_dim)
    out = torch.empty(M, n_q, head_dim, dtype=qkv.dtype, device=qkv.device)
    rep = n_q // n_kv
    cu = cu_seqlens.tolist()
    for i in range(len(cu) - 1):
        s, e = cu[i], cu[i + 1]
        if e <= s:
            continue
        qi = q[s:e].float().transpose(0, 1)  # [H, T, D]
        ki = k[s:e].float().transpose(0, 1).repeat_interleave(rep, 0)
        vi = v[s:e].float().transpose(0, 1).repeat_interleave(rep, 0)
        att = (qi @ ki.transpose(-1, -2)) * scale
        if causal:
            T = e - s
            mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
            att = att.masked_fill(~mask, float("-inf"))
        p = att.softmax(-1)
        out[s:e] = (p @ vi).transpose(0, 1).to(qkv.dtype)
    if cu[-1] < M:  # tokens outside any sequence (should not happen) -> zeros
        out[cu[-1]:] = 0
    return out.view(M, n_q * head_dim)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor):
    """Per-token CE in fp32 (ignore_index=-100). Returns (loss_per_token, lse, argmax_correct, entropy)."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = labels != IGNORE_INDEX
    safe = labels.clamp(min=0)
    tgt = lf.gather(-1, safe[:, None]).squeeze(-1)
    loss = torch.where(valid, lse - tgt, torch.zeros_like(lse))
    p = torch.softmax(lf, -1)
    entropy = lse - (p * lf).sum(-1)
    correct = (lf.argmax(-1) == labels) & valid
    return loss, lse, correct, entropy


def adamw_(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
           master: Optional[torch.Tensor], lr: float, beta1: float, beta2: float, eps: float,
           weight_decay: float, step: int, grad_scale: float = 1.0, sr_seed: int = 0, sr_offset: int = 0) -> None:
    """Decoupled-weight-decay Adam (torch.optim.AdamW semantics) on flat tensors, in place.

    Math in fp32 whatever the storage dtypes (twin of csrc/optim.hip adamw_kernel). bf16 storage
    (parameters without a master copy, and bf16 moments) is written with stochastic rounding when
    ``sr_seed`` is set — the same hash streams as the kernel, so CPU and GPU agree bit for bit on
    the rounding — and round-to-nearest otherwise."""
    w = master if master is not None else param.float()
    g = grad.float() * grad_scale
    m = exp_avg.float().mul_(beta1).add_(g, alpha=1 - beta1)
    v = exp_avg_sq.float().mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v / bc2).sqrt().add_(eps)
    w.mul_(1 - lr * weight_decay)
    w.addcdiv_(m, denom, value=-lr / bc1)
    sr = bool(sr_seed) and master is None
    for dst, src, s in ((exp_avg, m, _SEED_M), (exp_avg_sq, v, _SEED_V)):
        if dst.dtype == torch.bfloat16 and sr:
            dst.copy_(bf16_stochastic_round(src, (int(sr_seed) ^ s) & _M32, sr_offset))
        else:
            dst.copy_(src)
    if master is not None:
        param.copy_(master)
    elif sr and param.dtype == torch.bfloat16:
        param.copy_(bf16_stochastic_round(w, int(sr_seed), sr_offset))
    else:
        param.copy_(w)


_M32 = 0xFFFFFFFF
_SEED_M, _SEED_V = 0x68E31DA4, 0xB5297A4D  # csrc/optim.hip SEED_M / SEED_V


def hash_u32(idx: torch.Tensor, seed: int) -> torch.Tensor:
    """Bit-exact torch twin of csrc/common.h hash_u32 (int64 tensors holding uint32 values)."""
    lo, hi = idx & _M32, (idx >> 32) & _M32
    x = ((lo * 0x9E3779B9) & _M32) ^ ((hi * 0x85EBCA6B) & _M32) ^ ((int(seed) * 0xC2B2AE35) & _M32)
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def bf16_stochastic_round(x: torch.Tensor, seed: int, offset: int = 0) -> torch.Tensor:
    """fp32 -> bf16 with stochastic rounding: bits + noise(offset + i), truncated, where elements 2q / 2q + 1 take the
    low / high 16 bits of hash(q, seed). Twin of csrc/optim.hip f2bf_sr / sr_hash over a flat tensor (E[result] = x)."""
    xf = x.float().contiguous().reshape(-1)
    idx = torch.arange(xf.numel(), dtype=torch.int64, device=xf.device) + int(offset)
    bits = xf.view(torch.int32).to(torch.int64) & _M32
    finite = (bits & 0x7F800000) != 0x7F800000
    h = hash_u32(idx >> 1, seed)
    noise = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    rounded = ((bits + noise) >> 16) << 16
    out = torch.where(finite, rounded, bits)
    out = torch.where(out >= 1 << 31, out - (1 << 32), out).to(torch.int32).view(torch.float32)
    res = out.to(torch.bfloat16)  # exact: low 16 bits are zero (non-finite: round-to-nearest, as f2bf)
    return torch.where(finite, res, xf.to(torch.bfloat16)).view(x.shape)


def dropout_keep(idx: torch.Tensor, seed: int, p: float) -> torch.Tensor:
    """Twin of csrc/common.h drop_keep: elements 2q and 2q + 1 share hash(q, seed), whose low / high 16 bits are
    compared with int(p * 65536)."""
    h = hash_u32(idx >> 1, seed)
    half = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return half >= int(min(max(float(p), 0.0), 0.999) * 65536.0)


def dropout_add(a: Optional[torch.Tensor], b: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """(a or 0) + b * keep / (1-p), keep = dropout_keep(t*K + k) (same mask as the HIP kernels)."""
    T, K = b.shape
    p = min(max(float(p), 0.0), 0.999)
    idx = torch.arange(T * K, device=b.device, dtype=torch.int64).view(T, K)
    keep = dropout_keep(idx, seed, p)
    out = torch.where(keep, b.float() * (1.0 / (1.0 - p)), torch.zeros((), device=b.device))
    if a is not None:
        out = out + a.float()
    return out.to(b.dtype)


def lora_fwd(x: torch.Tensor, A: torch.Tensor, s: float, p: float, seed: int, ldX: int = 0):
    """(X' = [x | s * dropout(x) A^T | 0], xd = dropout(x) or None) — twin of csrc/lora.hip lora_fwd; ``ldX`` (0 =
    K + R) is the padded width of X'."""
    xd = dropout_add(None, x, p, seed) if p > 0 else None
    xa = (xd if xd is not None else x).float() @ A.float().t()
    parts = [x, (xa * s).to(x.dtype)]
    pad = (ldX or x.shape[1] + A.shape[0]) - x.shape[1] - A.shape[0]
    if pad > 0:
        parts.append(x.new_zeros(x.shape[0], pad))
    return torch.cat(parts, dim=1), xd


def lora_bwd_dx(base: torch.Tensor, dxa: torch.Tensor, A: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """dx = base + dropout(dxa @ A) (same mask as the forward) — twin of csrc/lora.hip lora_bwd_dx."""
    dxd = (dxa.float() @ A.float()).to(base.dtype)
    if p > 0:
        return dropout_add(base, dxd, p, seed)
    return (base.float() + dxd.float()).to(base.dtype)
