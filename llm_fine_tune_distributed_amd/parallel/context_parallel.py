"""Context parallelism: ring attention over a process group (SURVEY §5.7 stretch item, §2.5 "CP").

The reference caps sequences at 1024 tokens and has no sequence/context parallelism. This module
lets one long sequence span several GPUs. Each rank of a context-parallel (CP) group holds a
contiguous chunk of ``L`` tokens of every sequence in the batch:

* rank r holds positions ``[r L, (r + 1) L)``;
* its local packed layout is ``[B * L, (n_q + 2 n_kv) * D]`` with ``cu_seqlens = [0, L, 2L, ...]``.

Attention rotates the K/V chunks around the ring.

Forward (step s = 0 .. cp-1, holding the chunk of rank ``src = (r - s) mod cp``):
  * src == r: causal block;
  * src < r: full block, since every key precedes every query;
  * src > r: skipped (future keys).
  Each block is one call of the varlen flash-attention kernel (``csrc/attention.hip``) on the
  packed ``[q_local | kv_src]`` layout. It returns the block output and its log-sum-exp. The blocks
  are merged with the usual online-softmax rescaling in fp32. The send of the current chunk to rank
  r+1 and the receive from r-1 are posted before the block's compute, so the RCCL P2P transfer over
  xGMI overlaps the kernel.

Backward (FlashAttention-2 formulation): every block's gradient uses the FINAL output and
log-sum-exp, so the blocks are independent.
  * dQ accumulates locally.
  * dK/dV accumulate in fp32 buffers that travel around the ring with their K/V chunk. A final hop
    returns each buffer to its owner.

Model parameters are replicated across the CP group like data-parallel replicas. The DDP engine
sums gradients over the whole world, and the loss is normalised by the global token count
(``num_items_in_batch``), so the result equals single-GPU training on the full sequences. That is
tested in ``tests/test_context_parallel_cpu.py``. CPU tensors (gloo) take an fp32 PyTorch block
path with the same interface, which is what the CPU tests exercise.

Layouts (``layout=``):
* ``"zigzag"`` (default): every sequence is cut into 2 cp half-chunks and rank r holds half-chunks r and
  2 cp - 1 - r, concatenated. With causal attention every ring step then costs every rank exactly two
  (L/2)^2 blocks — (q_r, kv_src) and (q_{2cp-1-r}, kv_src) below the diagonal, or the two causal diagonal
  halves plus (q_{2cp-1-r}, kv_r) at step 0 — so no rank waits for another (the causal work of rank r is
  balanced; with contiguous chunks rank cp - 1 computes cp blocks and rank 0 one).
* ``"contiguous"``: rank r holds positions ``[r L, (r + 1) L)`` (simplest; unbalanced).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist
from torch.autograd import Function

from ..ops import _ext


# ----------------------------------------------------------------------------------------- blocks
def _block_fwd_ref(q, kv, cu, n_q, n_kv, D, scale, causal) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 reference block: (o [M, n_q D], lse [n_q, M]) of q against kv = [k | v] (GQA)."""
    M = q.shape[0]
    rep = n_q // n_kv
    qf = q.float().view(M, n_q, D)
    kf = kv[:, : n_kv * D].float().view(M, n_kv, D)
    vf = kv[:, n_kv * D:].float().view(M, n_kv, D)
    o = torch.zeros(M, n_q, D, dtype=torch.float32, device=q.device)
    lse = torch.full((n_q, M), -float("inf"), dtype=torch.float32, device=q.device)
    cl = cu.tolist()
    for i in range(len(cl) - 1):
        s, e = cl[i], cl[i + 1]
        if e <= s:
            continue
        qi = qf[s:e].transpose(0, 1)                               # [H, T, D]
        ki = kf[s:e].transpose(0, 1).repeat_interleave(rep, 0)
        vi = vf[s:e].transpose(0, 1).repeat_interleave(rep, 0)
        att = (qi @ ki.transpose(-1, -2)) * scale
        if causal:
            T = e - s
            att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=q.device).tril(), float("-inf"))
        l = torch.logsumexp(att, -1)                                # [H, T]
        o[s:e] = (torch.exp(att - l[..., None]) @ vi).transpose(0, 1)
        lse[:, s:e] = l
    return o.view(M, n_q * D), lse


def _block_bwd_ref(dout, q, kv, out, lse, cu, n_q, n_kv, D, scale, causal):
    """fp32 reference block backward given the FINAL out / lse: returns (dq [M, n_q D], dkv [M, 2 n_kv D])."""
    M = q.shape[0]
    rep = n_q // n_kv
    qf = q.float().view(M, n_q, D)
    kf = kv[:, : n_kv * D].float().view(M, n_kv, D)
    vf = kv[:, n_kv * D:].float().view(M, n_kv, D)
    of = out.float().view(M, n_q, D)
    df = dout.float().view(M, n_q, D)
    dq = torch.zeros(M, n_q, D, dtype=torch.float32, device=q.device)
    dk = torch.zeros(M, n_kv, D, dtype=torch.float32, device=q.device)
    dv = torch.zeros(M, n_kv, D, dtype=torch.float32, device=q.device)
    cl = cu.tolist()
    for i in range(len(cl) - 1):
        s, e = cl[i], cl[i + 1]
        if e <= s:
            continue
        T = e - s
        qi = qf[s:e].transpose(0, 1)
        ki = kf[s:e].transpose(0, 1).repeat_interleave(rep, 0)
        vi = vf[s:e].transpose(0, 1).repeat_interleave(rep, 0)
        oi, di = of[s:e].transpose(0, 1), df[s:e].transpose(0, 1)
        att = (qi @ ki.transpose(-1, -2)) * scale
        p = torch.exp(att - lse[:, s:e, None])
        if causal:
            p = p.masked_fill(~torch.ones(T, T, dtype=torch.bool, device=q.device).tril(), 0.0)
        dvi = p.transpose(-1, -2) @ di                              # [H, Tk, D]
        dp = di @ vi.transpose(-1, -2)
        delta = (di * oi).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dq[s:e] = ((ds @ ki) * scale).transpose(0, 1)
        dki = (ds.transpose(-1, -2) @ qi) * scale
        dk[s:e] = dki.view(n_kv, rep, T, D).sum(1).transpose(0, 1)
        dv[s:e] = dvi.view(n_kv, rep, T, D).sum(1).transpose(0, 1)
    return dq.view(M, n_q * D), torch.cat([dk.view(M, -1), dv.view(M, -1)], 1)


def _block_fwd(q, kv, cu, max_seqlen, n_q, n_kv, D, scale, causal):
    if _ext.use_hip(q):
        qkv = torch.cat([q, kv], 1).contiguous()
        o, lse = _ext.ops().flash_fwd(qkv, cu, max_seqlen, n_q, n_kv, D, scale, causal)
        return o.float(), lse
    return _block_fwd_ref(q, kv, cu, n_q, n_kv, D, scale, causal)


def _block_bwd(dout, q, kv, out, lse, cu, max_seqlen, n_q, n_kv, D, scale, causal):
    if _ext.use_hip(q):
        qkv = torch.cat([q, kv], 1).contiguous()
        d = _ext.ops().flash_bwd(dout, qkv, out, lse, cu, max_seqlen, n_q, n_kv, D, scale, causal)
        return d[:, : n_q * D].float(), d[:, n_q * D:].float()
    return _block_bwd_ref(dout, q, kv, out, lse, cu, n_q, n_kv, D, scale, causal)


def _merge(o, lse, o_s, lse_s, n_q, D):
    """Online-softmax merge of two partial attentions (fp32; lse [n_q, M], o [M, n_q D])."""
    if o is None:
        return o_s, lse_s
    new = torch.logaddexp(lse, lse_s)
    a = torch.exp(lse - new).t().unsqueeze(-1)                  # [M, n_q, 1]
    b = torch.exp(lse_s - new).t().unsqueeze(-1)
    M = o.shape[0]
    o = (o.view(M, n_q, D) * a + o_s.view(M, n_q, D) * b).view(M, n_q * D)
    return o, new


# ----------------------------------------------------------------------------------------- ring
def _ring_peers(group):
    ranks = dist.get_process_group_ranks(group)
    r = dist.get_rank(group)
    n = len(ranks)
    return r, n, ranks[(r + 1) % n], ranks[(r - 1) % n]


def _exchange(tensors, nxt, prv, group):
    """Post the send of ``tensors`` to ``nxt`` and the receive of same-shaped buffers from ``prv``."""
    bufs = [torch.empty_like(t) for t in tensors]
    ops = [dist.P2POp(dist.isend, t, nxt, group) for t in tensors]
    ops += [dist.P2POp(dist.irecv, b, prv, group) for b in bufs]
    return bufs, dist.batch_isend_irecv(ops)


class RingAttnFn(Function):
    """Contiguous layout: one causal / full block per ring step (see module docstring)."""

    @staticmethod
    def forward(ctx, qkv, cu, max_seqlen, n_q, n_kv, D, scale, group):
        r, n, nxt, prv = _ring_peers(group)
        q = qkv[:, : n_q * D]
        cur = qkv[:, n_q * D:].contiguous()
        o = lse = None
        for s in range(n):
            src = (r - s) % n
            pending = None
            if s < n - 1:
                (nxt_buf,), pending = _exchange([cur], nxt, prv, group)
            if src <= r:
                o_s, lse_s = _block_fwd(q, cur, cu, max_seqlen, n_q, n_kv, D, scale, causal=(src == r))
                o, lse = _merge(o, lse, o_s, lse_s, n_q, D)
            if pending is not None:
                for w in pending:
                    w.wait()
                cur = nxt_buf
        out = o.to(qkv.dtype)
        ctx.save_for_backward(qkv, cu, out, lse)
        ctx.dims = (max_seqlen, n_q, n_kv, D, scale)
        ctx.group = group
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, cu, out, lse = ctx.saved_tensors
        max_seqlen, n_q, n_kv, D, scale = ctx.dims
        group = ctx.group
        r, n, nxt, prv = _ring_peers(group)
        dout = dout.contiguous()
        q = qkv[:, : n_q * D]
        cur = qkv[:, n_q * D:].contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dkv = torch.zeros(cur.shape, dtype=torch.float32, device=q.device)
        for s in range(n):
            src = (r - s) % n
            # K/V for the next step can fly while this block computes; its dK/dV partner follows it
            pending_kv = None
            if s < n - 1:
                (nxt_kv,), pending_kv = _exchange([cur], nxt, prv, group)
            if src <= r:
                dq_s, dkv_s = _block_bwd(dout, q, cur, out, lse, cu, max_seqlen, n_q, n_kv, D, scale,
                                         causal=(src == r))
                dq += dq_s
                dkv += dkv_s
            (nxt_dkv,), pending = _exchange([dkv], nxt, prv, group)
            for w in pending + (pending_kv or []):
                w.wait()
            dkv = nxt_dkv  # after n hops every dK/dV buffer is back with the rank that owns its chunk
            if pending_kv is not None:
                cur = nxt_kv
        dqkv = torch.cat([dq, dkv], 1).to(qkv.dtype)
        return dqkv, None, None, None, None, None, None, None


def _zz_pairs(r: int, src: int, n: int):
    """(q half, kv half, causal) blocks of a zig-zag ring step: local half 0 / 1 of rank x is global
    half-chunk x / 2n - 1 - x; a key half-chunk below the query's is a full block, the same one causal."""
    qc = (r, 2 * n - 1 - r)
    kc = (src, 2 * n - 1 - src)
    out = []
    for x in range(2):
        for y in range(2):
            if kc[y] < qc[x]:
                out.append((x, y, False))
            elif kc[y] == qc[x]:
                out.append((x, y, True))
    return out


def _halves(t: torch.Tensor, B: int, h: int):
    """[B * 2h, F] -> the two [B * h, F] half-chunk row sets (copies)."""
    v = t.view(B, 2, h, t.shape[-1])
    return [v[:, 0].reshape(B * h, -1), v[:, 1].reshape(B * h, -1)]


def _join(a: torch.Tensor, b: torch.Tensor, B: int, h: int) -> torch.Tensor:
    return torch.stack([a.view(B, h, -1), b.view(B, h, -1)], 1).reshape(B * 2 * h, -1)


class ZigzagRingAttnFn(Function):
    """Zig-zag layout (module docstring): local rows are [half r | half 2n-1-r] per sequence of 2h tokens."""

    @staticmethod
    def forward(ctx, qkv, B, h, n_q, n_kv, D, scale, group):
        r, n, nxt, prv = _ring_peers(group)
        qh = _halves(qkv[:, : n_q * D], B, h)
        cur = qkv[:, n_q * D:].contiguous()
        cu = torch.arange(0, (B + 1) * h, h, dtype=torch.int32, device=qkv.device)
        o = [None, None]
        lse = [None, None]
        for s in range(n):
            src = (r - s) % n
            pending = None
            if s < n - 1:
                (nxt_buf,), pending = _exchange([cur], nxt, prv, group)
            kvh = _halves(cur, B, h)
            for x, y, causal in _zz_pairs(r, src, n):
                o_s, lse_s = _block_fwd(qh[x], kvh[y], cu, h, n_q, n_kv, D, scale, causal=causal)
                o[x], lse[x] = _merge(o[x], lse[x], o_s, lse_s, n_q, D)
            if pending is not None:
                for w in pending:
                    w.wait()
                cur = nxt_buf
        out = _join(o[0], o[1], B, h).to(qkv.dtype)
        ctx.save_for_backward(qkv, out, lse[0], lse[1])
        ctx.dims = (B, h, n_q, n_kv, D, scale)
        ctx.group = group
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse0, lse1 = ctx.saved_tensors
        B, h, n_q, n_kv, D, scale = ctx.dims
        group = ctx.group
        r, n, nxt, prv = _ring_peers(group)
        qh = _halves(qkv[:, : n_q * D], B, h)
        oh = _halves(out, B, h)
        dh = _halves(dout.contiguous(), B, h)
        lse = (lse0, lse1)
        cu = torch.arange(0, (B + 1) * h, h, dtype=torch.int32, device=qkv.device)
        cur = qkv[:, n_q * D:].contiguous()
        dq = [torch.zeros(B * h, n_q * D, dtype=torch.float32, device=qkv.device) for _ in range(2)]
        dkv = torch.zeros(cur.shape, dtype=torch.float32, device=qkv.device)
        for s in range(n):
            src = (r - s) % n
            pending_kv = None
            if s < n - 1:
                (nxt_kv,), pending_kv = _exchange([cur], nxt, prv, group)
            kvh = _halves(cur, B, h)
            dkvh = [torch.zeros(B * h, cur.shape[1], dtype=torch.float32, device=qkv.device) for _ in range(2)]
            for x, y, causal in _zz_pairs(r, src, n):
                dq_s, dkv_s = _block_bwd(dh[x], qh[x], kvh[y], oh[x], lse[x], cu, h, n_q, n_kv, D, scale,
                                         causal=causal)
                dq[x] += dq_s
                dkvh[y] += dkv_s
            dkv = dkv + _join(dkvh[0], dkvh[1], B, h)
            (nxt_dkv,), pending = _exchange([dkv], nxt, prv, group)
            for w in pending + (pending_kv or []):
                w.wait()
            dkv = nxt_dkv
            if pending_kv is not None:
                cur = nxt_kv
        dqkv = torch.cat([_join(dq[0], dq[1], B, h), dkv], 1).to(qkv.dtype)
        return dqkv, None, None, None, None, None, None, None


def ring_attention(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, group, scale: Optional[float] = None,
                   layout: str = "zigzag"):
    """Causal GQA attention for a sequence-sharded batch (see module docstring); ``qkv`` is this rank's
    packed chunk [B * L, (n_q + 2 n_kv) * D], ``cu_seqlens`` its local sequence boundaries (equal lengths L;
    zig-zag: L even, rows [half r | half 2 cp - 1 - r] per sequence)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if group is None or dist.get_world_size(group) == 1:
        from ..ops import flash_attention
        return flash_attention(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, True)
    if layout == "zigzag":
        L = int(max_seqlen)
        B = qkv.shape[0] // L
        if L % 2 or B * L != qkv.shape[0]:
            raise ValueError("zig-zag context parallelism needs equal, even local sequence lengths")
        return ZigzagRingAttnFn.apply(qkv, B, L // 2, n_q, n_kv, head_dim, scale, group)
    return RingAttnFn.apply(qkv, cu_seqlens, max_seqlen, n_q, n_kv, head_dim, scale, group)


# ----------------------------------------------------------------------------------------- data
def shard_batch(b: Dict, cp_rank: int, cp_size: int, pad_id: int = 0, layout: str = "zigzag") -> Dict:
    """Cut a padded micro-batch ([B, T] input_ids / labels, unshifted HF labels) into this CP rank's chunk.

    Labels are shifted over the FULL sequence first (the last token of chunk r is scored against the
    first token of chunk r + 1), T is padded to a multiple of ``cp_size`` (zig-zag: ``2 cp_size``; pads:
    ``pad_id`` / -100), and the chunk carries its global ``position_ids`` so RoPE sees the true positions.
    ``num_items`` becomes the local count of scored tokens: summed over every rank it is the global count the
    loss is normalised by. Zig-zag: the chunk is half-chunks cp_rank and 2 cp_size - 1 - cp_rank."""
    ids, labels = b["input_ids"], b["labels"]
    if ids.dim() != 2 or "cu_seqlens" in b:
        raise ValueError("context parallelism expects padded [B, T] batches (packing=False)")
    B, T = ids.shape
    shifted = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], -100)], dim=1)
    unit = 2 * cp_size if layout == "zigzag" else cp_size
    Tp = -(-T // unit) * unit
    if Tp != T:
        ids = torch.cat([ids, torch.full((B, Tp - T), pad_id, dtype=ids.dtype, device=ids.device)], 1)
        shifted = torch.cat([shifted, torch.full((B, Tp - T), -100, dtype=shifted.dtype, device=shifted.device)], 1)
    if layout == "zigzag":
        h = Tp // (2 * cp_size)
        pos = torch.cat([torch.arange(cp_rank * h, (cp_rank + 1) * h),
                         torch.arange((2 * cp_size - 1 - cp_rank) * h, (2 * cp_size - cp_rank) * h)]).to(ids.device)
    else:
        L = Tp // cp_size
        pos = torch.arange(cp_rank * L, (cp_rank + 1) * L, device=ids.device)
    out = dict(b)
    out["input_ids"] = ids[:, pos].contiguous()
    out["labels"] = shifted[:, pos].contiguous()
    out["shifted"] = True
    out["position_ids"] = pos.expand(B, pos.numel())
    n = int((out["labels"] != -100).sum())
    out["num_items"] = n
    out["num_items_t"] = torch.tensor([float(n)], device=ids.device)
    return out


def new_groups(world_size: int, rank: int, cp_size: int):
    """Partition the world into consecutive CP groups of ``cp_size`` ranks (every rank creates every group,
    as torch.distributed requires). Returns (cp_group, cp_rank, dp_rank, dp_size)."""
    if cp_size < 1 or world_size % cp_size:
        raise ValueError(f"context_parallel_size {cp_size} must divide world_size {world_size}")
    mine = None
    for g in range(world_size // cp_size):
        ranks = list(range(g * cp_size, (g + 1) * cp_size))
        pg = dist.new_group(ranks)
        if rank in ranks:
            mine = pg
    return mine, rank % cp_size, rank // cp_size, world_size // cp_size
