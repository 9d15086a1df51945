"""Decoder-only causal LM (SmolLM3 / Llama family) built on the fused ops.

Replaces ``AutoModelForCausalLM.from_pretrained(...)`` of the reference
(``training.py:97-105``) and the transformers modules it runs
(``transformers/models/smollm3/modeling_smollm3.py``).

MI355X-first layout decisions:
* tokens are packed as a flat [M = sum(len), hidden] stream; attention is varlen over
  ``cu_seqlens`` so padded batches and padding-free packing share one code path;
* q/k/v and gate/up are fused weights (one GEMM each); HF key names are restored on
  save/load (``hf_state_dict`` / ``load_hf_state_dict``);
* RoPE is applied in place on the packed qkv GEMM output, NoPE layers skip it;
* the LM head and cross-entropy are one op that never materialises fp32 logits.
"""
from __future__ import annotations

import math
import os
import zlib
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from .. import ops
from ..ops import reference as ref
from .config import ModelConfig


@dataclass
class CausalLMOutput:
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = None
    stats: Optional[torch.Tensor] = None  # [4, M]: loss, lse, entropy, correct (per token)
    num_tokens: Optional[torch.Tensor] = None
    metrics: Optional[torch.Tensor] = None


class RMSNorm(nn.Module):
    def __init__(self, hidden: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden))
        self.eps = eps


class Attention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int):
        super().__init__()
        self.cfg = cfg
        self.layer_idx = layer_idx
        self.use_rope = cfg.uses_rope(layer_idx)
        self.qkv_proj = nn.Parameter(torch.empty(cfg.qkv_size, cfg.hidden_size))
        self.o_proj = nn.Parameter(torch.empty(cfg.hidden_size, cfg.q_size))
        self.lora = None  # set by apply_lora
        self.cp_group = None  # context-parallel process group (CausalLM.enable_context_parallel)
        self.cp_layout = "zigzag"

    def forward(self, h, rope_cs, cu_seqlens, max_seqlen):
        c = self.cfg
        if self.lora is None and self.use_rope and self.cp_group is None:
            # projection + RoPE (GEMM epilogue) + attention as one autograd node: the backward applies the inverse
            # rotation inside the attention kernels' dq / dK epilogues
            # the o_proj backward computes the attention backward's delta in its dgrad epilogue (box: the hand-off)
            box = {}
            a = ops.qkv_rope_attention(h, self.qkv_proj, rope_cs[0], rope_cs[1], cu_seqlens, max_seqlen,
                                       c.num_attention_heads, c.num_key_value_heads, c.head_dim, delta_box=box)
            return ops.attn_out_linear(a, self.o_proj, box)
        if self.lora is not None and self.use_rope and self.cp_group is None:
            # the LoRA-widened qkv GEMM with the RoPE epilogue + attention as one node (inverse RoPE in the backward's
            # dq / dK epilogues), the plain composition where the HIP path does not apply
            a = ops.lora_qkv_rope_attention(h, self.qkv_proj, self.lora["qkv"], rope_cs[0], rope_cs[1], cu_seqlens,
                                            max_seqlen, c.num_attention_heads, c.num_key_value_heads, c.head_dim)
            return ops.lora_linear(a, self.o_proj, self.lora["o"])
        pair = None
        if self.lora is None and self.use_rope:
            # projection + RoPE in one HIP GEMM (epilogue rotation) where the shapes allow
            qkv = ops.linear_rope(h, self.qkv_proj, rope_cs[0], rope_cs[1], c.num_attention_heads,
                                  c.num_key_value_heads, c.head_dim)
        else:
            # (a NoPE layer: the qkv node also issues o_proj's weight gradient, as one launch with its own)
            pair = {} if (self.lora is None and not self.use_rope and self.cp_group is None) else None
            qkv = (ops.qkv_in_linear(h, self.qkv_proj, pair) if self.lora is None
                   else ops.lora_linear(h, self.qkv_proj, self.lora["qkv"]))
            if self.use_rope:
                qkv = ops.rope_(qkv, rope_cs[0], rope_cs[1], c.num_attention_heads, c.num_key_value_heads, c.head_dim)
        if self.cp_group is not None:
            from ..parallel.context_parallel import ring_attention
            a = ring_attention(qkv, cu_seqlens, max_seqlen, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                               self.cp_group, layout=self.cp_layout)
        else:
            box = (pair if pair is not None else {}) if self.lora is None else None
            a = ops.flash_attention(qkv, cu_seqlens, max_seqlen, c.num_attention_heads, c.num_key_value_heads,
                                    c.head_dim, delta_box=box)
            if box is not None:
                return ops.attn_out_linear(a, self.o_proj, box)
        return ops.linear(a, self.o_proj) if self.lora is None else ops.lora_linear(a, self.o_proj, self.lora["o"])


class MLP(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.gate_up_proj = nn.Parameter(torch.empty(2 * cfg.intermediate_size, cfg.hidden_size))
        self.down_proj = nn.Parameter(torch.empty(cfg.hidden_size, cfg.intermediate_size))
        self.lora = None

    def forward(self, h):
        L = self.lora
        if L is None:  # SwiGLU fused into the GEMM epilogues where the kernels apply (ops.swiglu_mlp)
            return ops.swiglu_mlp(h, self.gate_up_proj, self.down_proj)
        return ops.lora_swiglu_mlp(h, self.gate_up_proj, self.down_proj, L["gate_up"], L["down"])


def _wide_ld(lora, key: str, weight) -> int:
    """Row width of the LoRA wide weight W' that consumes this norm's output (0: none), so the norm writes its output
    straight into the left block of the consumer's widened activation X' (ops.add_rms_norm y_ld)."""
    fl = None if lora is None else lora[key]
    wide = getattr(fl, "wide", None)
    if wide is None or not any(fl.active) or weight.data_ptr() != wide.data_ptr():
        return 0
    # only where the consumer's in-place widening kernel takes the shape (else the norm writes a plain y and the
    # consumer copies it into X')
    if not ops.lora_inplace_ok(fl.in_features, fl.r * sum(1 for a in fl.active if a)):
        return 0
    return wide.shape[1]


class DecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = Attention(cfg, layer_idx)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = MLP(cfg)

    def forward(self, x, residual, rope_cs, cu_seqlens, max_seqlen):
        """Pre-norm block with the residual add fused into the norms:
        (x: previous sublayer output, residual: residual stream before adding x)."""
        ln = self.input_layernorm
        at, ml = self.self_attn, self.mlp
        h, residual = ops.add_rms_norm(x, residual, ln.weight, ln.eps, _wide_ld(at.lora, "qkv", at.qkv_proj))
        a = at(h, rope_cs, cu_seqlens, max_seqlen)
        ln2 = self.post_attention_layernorm
        h, residual = ops.add_rms_norm(a, residual, ln2.weight, ln2.eps, _wide_ld(ml.lora, "gate_up", ml.gate_up_proj))
        return ml(h), residual


class Model(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.embed_tokens = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size))
        self.layers = nn.ModuleList([DecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)


class CausalLM(nn.Module):
    """SmolLM3ForCausalLM / LlamaForCausalLM equivalent."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.config = cfg
        self.model = Model(cfg)
        if cfg.tie_word_embeddings:
            self.lm_head = None
        else:
            self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size))
        self.gradient_checkpointing = False
        inv = ref.rope_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.register_buffer("inv_freq", inv, persistent=False)
        self._declare_uses()

    # ------------------------------------------------------------------ params
    @property
    def lm_head_weight(self) -> torch.Tensor:
        return self.model.embed_tokens if self.lm_head is None else self.lm_head

    def _declare_uses(self):
        for p in self.parameters():
            p._sftamd_uses = 1
        if self.lm_head is None:
            self.model.embed_tokens._sftamd_uses = 2

    def reset_grad_use_counters(self):
        for p in self.parameters():
            if p.requires_grad:
                p._sftamd_remaining = getattr(p, "_sftamd_uses", 1)

    def gradient_checkpointing_enable(self, **_):
        self.gradient_checkpointing = True

    def gradient_checkpointing_disable(self):
        self.gradient_checkpointing = False

    def enable_context_parallel(self, group, layout: str = "zigzag") -> None:
        """Attention over sequence chunks spread across ``group`` (ring attention, parallel/context_parallel.py).
        Inputs must then be this rank's chunk with explicit global ``position_ids`` and pre-shifted labels
        (``context_parallel.shard_batch`` with the same ``layout``)."""
        for layer in self.model.layers:
            layer.self_attn.cp_group = group
            layer.self_attn.cp_layout = layout

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Random init (HF-style normal(0, initializer_range), norms = 1). Deterministic per seed
        so every DDP rank builds identical weights without a 6 GB broadcast."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        std = self.config.initializer_range
        for name, p in self.named_parameters():
            if name.endswith("layernorm.weight") or name.endswith("norm.weight"):
                p.fill_(1.0)
            elif p.device.type == "cpu":
                p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float32).mul_(std).to(p.dtype))
            else:
                gg = torch.Generator(device=p.device).manual_seed(seed * 1000003 + zlib.crc32(name.encode()))
                p.normal_(0.0, std, generator=gg)
        return self

    def num_parameters(self, trainable_only: bool = False) -> int:
        seen, n = set(), 0
        for p in self.parameters():
            if id(p) in seen or (trainable_only and not p.requires_grad):
                continue
            seen.add(id(p))
            n += p.numel()
        return n

    # ------------------------------------------------------------------ forward
    def _padded_meta(self, B: int, T: int, dev):
        cache = self.__dict__.setdefault("_meta_cache", {})
        key = (B, T, str(dev), self.inv_freq.data_ptr())
        hit = cache.get(key)
        if hit is None:
            if len(cache) >= 8:
                cache.clear()
            cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device=dev)
            hit = cache[key] = (cu, T, self.rope_tables(torch.arange(T, device=dev).expand(B, T)))
        return hit

    def rope_tables(self, position_ids: torch.Tensor):
        freqs = position_ids.reshape(-1).float()[:, None] * self.inv_freq[None, :].to(position_ids.device)
        return freqs.cos().contiguous(), freqs.sin().contiguous()

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None,
                cu_seqlens: Optional[torch.Tensor] = None, max_seqlen: Optional[int] = None,
                position_ids: Optional[torch.Tensor] = None, num_items_in_batch=None,
                return_logits: bool = False, shift_labels: bool = True, **_) -> CausalLMOutput:
        """input_ids [B, T] (padded, right) or [M] (packed with cu_seqlens).

        ``labels`` are unshifted HF-style labels (-100 ignored) unless ``shift_labels=False``.
        Loss = sum of token CE / num_items_in_batch (HF ``num_items_in_batch`` semantics), or the
        mean over valid tokens when ``num_items_in_batch`` is None.
        """
        cfg = self.config
        dev = input_ids.device
        rope_cs = None
        if input_ids.dim() == 2 and cu_seqlens is None and position_ids is None:
            # padded batches of one shape repeat every step: cu_seqlens / RoPE tables are built once
            cu_seqlens, max_seqlen, rope_cs = self._padded_meta(input_ids.shape[0], input_ids.shape[1], dev)
        if input_ids.dim() == 2:
            B, T = input_ids.shape
            if cu_seqlens is None:
                cu_seqlens = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device=dev)
                max_seqlen = T
            if position_ids is None:
                position_ids = torch.arange(T, device=dev).expand(B, T)
            if labels is not None and shift_labels:
                labels = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], -100)], dim=1)
                shift_labels = False
        ids = input_ids.reshape(-1)
        M = ids.numel()
        if cu_seqlens is None:
            cu_seqlens = torch.tensor([0, M], dtype=torch.int32, device=dev)
            max_seqlen = M
        if max_seqlen is None:
            max_seqlen = int((cu_seqlens[1:] - cu_seqlens[:-1]).max().item())
        if position_ids is None:
            position_ids = _positions_from_cu(cu_seqlens, M)
        if labels is not None:
            labels = labels.reshape(-1)
            if shift_labels:
                labels = _shift_packed(labels, cu_seqlens)
        if rope_cs is None:
            rope_cs = self.rope_tables(position_ids)

        x = ops.embedding(ids, self.model.embed_tokens)
        residual = None
        ckpt = self.gradient_checkpointing and self.training and torch.is_grad_enabled()
        # (a layer's o_proj + qkv weight gradients join the previous layer's MLP launch: ops.wgrad_carry_scope)
        with ops.wgrad_carry_scope(enabled=not ckpt):
            for layer in self.model.layers:
                if ckpt:
                    x, residual = checkpoint(layer, x, residual, rope_cs, cu_seqlens, max_seqlen, use_reentrant=False)
                else:
                    x, residual = layer(x, residual, rope_cs, cu_seqlens, max_seqlen)
        n = self.model.norm
        h, _ = ops.add_rms_norm(x, residual, n.weight, n.eps)

        out = CausalLMOutput()
        if labels is not None:
            valid = labels != -100
            if hasattr(num_items_in_batch, "resolve"):  # trainer's in-flight global count (PendingCount)
                num_items_in_batch = num_items_in_batch.resolve()
            if num_items_in_batch is None:
                cnt = valid.sum().clamp(min=1)
            elif torch.is_tensor(num_items_in_batch):
                cnt = num_items_in_batch
            else:
                cnt = torch.tensor(float(num_items_in_batch))
            inv = (1.0 / cnt.to(device=dev, dtype=torch.float32)).reshape(1)
            out.loss, out.stats = ops.lm_head_cross_entropy(h, self.lm_head_weight, labels, inv)
            vf = valid.float()
            out.num_tokens = vf.sum()
            # TRL-style training metrics from the same fused CE pass: [correct, entropy_sum, valid]
            out.metrics = torch.stack([out.stats[3].sum(), (out.stats[2] * vf).sum(), out.num_tokens])
        if return_logits or labels is None:
            out.logits = torch.nn.functional.linear(h, self.lm_head_weight)
        return out

    # ------------------------------------------------------------------ HF state dict
    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """State dict with HF key names (q/k/v and gate/up split, tied lm_head omitted)."""
        cfg = self.config
        sd = {"model.embed_tokens.weight": self.model.embed_tokens.detach()}
        for i, l in enumerate(self.model.layers):
            p = f"model.layers.{i}."
            q, k, v = l.self_attn.qkv_proj.detach().split([cfg.q_size, cfg.kv_size, cfg.kv_size], 0)
            sd[p + "self_attn.q_proj.weight"] = q
            sd[p + "self_attn.k_proj.weight"] = k
            sd[p + "self_attn.v_proj.weight"] = v
            sd[p + "self_attn.o_proj.weight"] = l.self_attn.o_proj.detach()
            g, u = l.mlp.gate_up_proj.detach().split([cfg.intermediate_size] * 2, 0)
            sd[p + "mlp.gate_proj.weight"] = g
            sd[p + "mlp.up_proj.weight"] = u
            sd[p + "mlp.down_proj.weight"] = l.mlp.down_proj.detach()
            sd[p + "input_layernorm.weight"] = l.input_layernorm.weight.detach()
            sd[p + "post_attention_layernorm.weight"] = l.post_attention_layernorm.weight.detach()
        sd["model.norm.weight"] = self.model.norm.weight.detach()
        if self.lm_head is not None:
            sd["lm_head.weight"] = self.lm_head.detach()
        return sd

    @torch.no_grad()
    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        cfg = self.config
        used = set()

        def take(key):
            used.add(key)
            return sd[key]

        self.model.embed_tokens.copy_(take("model.embed_tokens.weight"))
        for i, l in enumerate(self.model.layers):
            p = f"model.layers.{i}."
            l.self_attn.qkv_proj.copy_(torch.cat([take(p + "self_attn.q_proj.weight"),
                                                  take(p + "self_attn.k_proj.weight"),
                                                  take(p + "self_attn.v_proj.weight")], 0))
            l.self_attn.o_proj.copy_(take(p + "self_attn.o_proj.weight"))
            l.mlp.gate_up_proj.copy_(torch.cat([take(p + "mlp.gate_proj.weight"), take(p + "mlp.up_proj.weight")], 0))
            l.mlp.down_proj.copy_(take(p + "mlp.down_proj.weight"))
            l.input_layernorm.weight.copy_(take(p + "input_layernorm.weight"))
            l.post_attention_layernorm.weight.copy_(take(p + "post_attention_layernorm.weight"))
        self.model.norm.weight.copy_(take("model.norm.weight"))
        if self.lm_head is not None:
            self.lm_head.copy_(take("lm_head.weight"))
        extra = set(sd) - used - {"lm_head.weight"}
        if strict and extra:
            raise KeyError(f"unexpected keys: {sorted(extra)[:8]}")
        return self


def _positions_from_cu(cu: torch.Tensor, M: int) -> torch.Tensor:
    idx = torch.arange(M, device=cu.device)
    seq = torch.searchsorted(cu[1:].to(torch.int64), idx, right=True)
    return idx - cu.to(torch.int64)[seq.clamp(max=cu.numel() - 2)]


def _shift_packed(labels: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
    out = torch.cat([labels[1:], labels.new_full((1,), -100)])
    ends = cu[1:].to(torch.int64) - 1
    ends = ends[ends >= 0]
    out[ends] = -100
    return out


def build_model(cfg: ModelConfig, device="cpu", dtype=torch.bfloat16, seed: int = 0) -> CausalLM:
    with torch.device("meta"):
        m = CausalLM(cfg)
    m = m.to_empty(device=device)
    m.inv_freq = ref.rope_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling, device=device)
    for p in m.parameters():
        p.data = p.data.to(dtype)
    m._declare_uses()
    m.init_weights(seed)
    return m
