"""KV-cache text generation (reference I1/I2: ``model.generate`` in ask_tuned_model.py:55-65).

Prefill runs the training kernels (fused RMSNorm, packed QKV GEMM, in-place RoPE, the varlen
flash-attention forward) over the prompt and stores K/V in a preallocated cache sized for the
whole generation (288 GB of HBM: no paging needed at this scale). Decode appends one token per
step; single-query GQA attention over the cache is a memory-bound GEMV (batched matmul on the
cache slice). Sampling matches HF's logits-processor order: repetition penalty -> temperature ->
top-k -> top-p -> multinomial.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from .. import ops


class KVCache:
    def __init__(self, cfg, max_len: int, device, dtype=torch.bfloat16):
        L = cfg.num_hidden_layers
        self.k = torch.empty(L, max_len, cfg.num_key_value_heads, cfg.head_dim, device=device, dtype=dtype)
        self.v = torch.empty_like(self.k)
        self.len = 0


@torch.no_grad()
def _layer(model, li, x, residual, cache: KVCache, pos: torch.Tensor, prefill: bool):
    cfg = model.config
    layer = model.model.layers[li]
    at = layer.self_attn
    nq, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    h, residual = ops.add_rms_norm(x, residual, layer.input_layernorm.weight, cfg.rms_norm_eps)
    qkv = ops.linear(h, at.qkv_proj) if at.lora is None else ops.lora_linear(h, at.qkv_proj, at.lora["qkv"])
    if at.use_rope:
        cos, sin = model.rope_tables(pos)
        ops.rope_(qkv, cos, sin, nq, nkv, D)
    M = qkv.shape[0]
    k = qkv[:, nq * D:(nq + nkv) * D].view(M, nkv, D)
    v = qkv[:, (nq + nkv) * D:].view(M, nkv, D)
    s = cache.len
    cache.k[li, s:s + M] = k
    cache.v[li, s:s + M] = v
    if prefill:
        cu = torch.tensor([0, M], dtype=torch.int32, device=x.device)
        a = ops.flash_attention(qkv.contiguous(), cu, M, nq, nkv, D)
    else:
        q = qkv[:, :nq * D].view(nq, D).float()
        K = cache.k[li, :s + 1].float()  # [S, nkv, D]
        V = cache.v[li, :s + 1].float()
        rep = nq // nkv
        qg = q.view(nkv, rep, D)
        att = torch.einsum("grd,sgd->grs", qg, K) / math.sqrt(D)
        p = att.softmax(-1)
        a = torch.einsum("grs,sgd->grd", p, V).reshape(1, nq * D).to(x.dtype)
    o = ops.linear(a, at.o_proj) if at.lora is None else ops.lora_linear(a, at.o_proj, at.lora["o"])
    h, residual = ops.add_rms_norm(o, residual, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
    return layer.mlp(h), residual


@torch.no_grad()
def forward_cached(model, ids: torch.Tensor, cache: KVCache, prefill: bool) -> torch.Tensor:
    """ids: [M] tokens appended at positions cache.len ... Returns last-token logits [V] (fp32)."""
    M = ids.numel()
    pos = torch.arange(cache.len, cache.len + M, device=ids.device)
    x = ops.embedding(ids, model.model.embed_tokens)
    residual = None
    for li in range(model.config.num_hidden_layers):
        x, residual = _layer(model, li, x, residual, cache, pos, prefill)
    cache.len += M
    n = model.model.norm
    h, _ = ops.add_rms_norm(x[-1:], residual[-1:], n.weight, model.config.rms_norm_eps)
    return torch.nn.functional.linear(h, model.lm_head_weight).float()[0]


def sample_next(logits: torch.Tensor, history: torch.Tensor, temperature: float = 0.6, top_k: int = 40,
                top_p: float = 0.95, repetition_penalty: float = 1.1, do_sample: bool = True,
                generator: Optional[torch.Generator] = None) -> int:
    logits = logits.clone()
    if repetition_penalty and repetition_penalty != 1.0 and history.numel():
        sc = logits[history]
        logits[history] = torch.where(sc < 0, sc * repetition_penalty, sc / repetition_penalty)
    if not do_sample:
        return int(logits.argmax())
    logits = logits / max(temperature, 1e-5)
    if top_k and top_k > 0:
        kth = torch.topk(logits, min(top_k, logits.numel())).values[-1]
        logits[logits < kth] = -float("inf")
    if top_p is not None and top_p < 1.0:
        sl, si = torch.sort(logits, descending=True)
        cp = sl.softmax(-1).cumsum(-1)
        remove = cp > top_p
        remove[1:] = remove[:-1].clone()
        remove[0] = False
        logits[si[remove]] = -float("inf")
    p = logits.softmax(-1)
    return int(torch.multinomial(p, 1, generator=generator))


@torch.no_grad()
def generate(model, prompt_ids: List[int], max_new_tokens: int = 256, eos_token_id: Optional[int] = None,
             temperature: float = 0.6, top_k: int = 40, top_p: float = 0.95, repetition_penalty: float = 1.1,
             do_sample: bool = True, seed: Optional[int] = None) -> List[int]:
    model.eval()
    dev = model.model.embed_tokens.device
    cache = KVCache(model.config, len(prompt_ids) + max_new_tokens + 1, dev, model.model.embed_tokens.dtype)
    g = torch.Generator(device=dev).manual_seed(seed) if seed is not None else None
    ids = torch.tensor(prompt_ids, device=dev)
    logits = forward_cached(model, ids, cache, prefill=True)
    hist = ids.clone()
    out: List[int] = []
    for _ in range(max_new_tokens):
        t = sample_next(logits, hist, temperature, top_k, top_p, repetition_penalty, do_sample, g)
        out.append(t)
        if eos_token_id is not None and t == eos_token_id:
            break
        nt = torch.tensor([t], device=dev)
        hist = torch.cat([hist, nt])
        logits = forward_cached(model, nt, cache, prefill=False)
    return out
