"""LoRA adapters on the fused projections (BASELINE.json config "LoRA SFT bf16 on 1xMI355X").

Defaults follow the Red Hat article shipped with the reference (external-doc docx¶64-72):
r=16, lora_alpha=8, dropout 0.05, all seven projections (q,k,v,o,gate,up,down).
The fused qkv / gate_up weights get one adapter per HF sub-projection, so the adapter
math (and saved keys) equals per-projection PEFT LoRA.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List

import torch
import torch.nn as nn

ALL_PROJ = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


@dataclass
class LoRAConfig:
    r: int = 16
    lora_alpha: float = 8.0
    lora_dropout: float = 0.05
    target_modules: List[str] = field(default_factory=lambda: list(ALL_PROJ))

    @property
    def scaling(self) -> float:
        return self.lora_alpha / self.r


class FusedLoRA(nn.Module):
    """delta(x) = concat_i(B_i A_i dropout(x)) * alpha/r over the sub-projections of a fused weight."""

    def __init__(self, in_features: int, out_splits: List[int], names: List[str], cfg: LoRAConfig,
                 active: List[bool], device=None, dtype=None):
        super().__init__()
        self.names = names
        self.in_features = in_features
        self.out_splits = out_splits
        self.active = active
        self.r = cfg.r
        self.scaling = cfg.scaling
        self.dropout = nn.Dropout(cfg.lora_dropout) if cfg.lora_dropout > 0 else nn.Identity()
        self.A = nn.ParameterList()
        self.B = nn.ParameterList()
        for n, act in zip(out_splits, active):
            a = torch.empty(cfg.r if act else 0, in_features, device=device, dtype=dtype)
            nn.init.kaiming_uniform_(a, a=math.sqrt(5)) if act else None
            self.A.append(nn.Parameter(a))
            self.B.append(nn.Parameter(torch.zeros(n, cfg.r if act else 0, device=device, dtype=dtype)))

    def forward(self, x):
        x = self.dropout(x)
        outs = []
        for a, b, n, act in zip(self.A, self.B, self.out_splits, self.active):
            if act:
                outs.append(torch.nn.functional.linear(torch.nn.functional.linear(x, a), b))
            else:
                outs.append(x.new_zeros(*x.shape[:-1], n))
        return torch.cat(outs, dim=-1) * self.scaling

    @torch.no_grad()
    def delta_weight(self) -> torch.Tensor:
        ws = []
        for a, b, n, act in zip(self.A, self.B, self.out_splits, self.active):
            ws.append((b.float() @ a.float()) if act else torch.zeros(n, self.in_features, device=a.device))
        return torch.cat(ws, 0) * self.scaling


def apply_lora(model, cfg: LoRAConfig = None):
    """Freeze the base model and attach adapters. Returns the model."""
    cfg = cfg or LoRAConfig()
    mc = model.config
    for p in model.parameters():
        p.requires_grad_(False)
    t = set(cfg.target_modules)
    ref_w = model.model.embed_tokens
    dev, dt = ref_w.device, ref_w.dtype
    for layer in model.model.layers:
        at, mlp = layer.self_attn, layer.mlp
        at.lora = nn.ModuleDict({
            "qkv": FusedLoRA(mc.hidden_size, [mc.q_size, mc.kv_size, mc.kv_size], ["q_proj", "k_proj", "v_proj"], cfg,
                             [n in t for n in ("q_proj", "k_proj", "v_proj")], dev, dt),
            "o": FusedLoRA(mc.q_size, [mc.hidden_size], ["o_proj"], cfg, ["o_proj" in t], dev, dt),
        })
        mlp.lora = nn.ModuleDict({
            "gate_up": FusedLoRA(mc.hidden_size, [mc.intermediate_size] * 2, ["gate_proj", "up_proj"], cfg,
                                 ["gate_proj" in t, "up_proj" in t], dev, dt),
            "down": FusedLoRA(mc.intermediate_size, [mc.hidden_size], ["down_proj"], cfg, ["down_proj" in t], dev, dt),
        })
    for n, p in model.named_parameters():
        if ".lora." in n and p.numel() > 0:
            p.requires_grad_(True)
    for layer in model.model.layers:
        for owner, wname, key in ((layer.self_attn, "qkv_proj", "qkv"), (layer.self_attn, "o_proj", "o"),
                                  (layer.mlp, "gate_up_proj", "gate_up"), (layer.mlp, "down_proj", "down")):
            _widen(owner, wname, owner.lora[key])
    model._lora_config = cfg
    return model


@torch.no_grad()
def _widen(owner: nn.Module, wname: str, fl: FusedLoRA) -> None:
    """Re-home the frozen base weight W [n, K] as the left block of W' = [W | B_blockdiag | 0] [n, K+Rp]
    (ops.LoRAWideFn): the base Parameter becomes a column-slice view of W', so checkpoint I/O,
    merge_lora and plain inference keep working on it unchanged."""
    w = getattr(owner, wname)
    act = [i for i, a in enumerate(fl.active) if a]
    if not act:
        return
    n, K = w.shape
    R = fl.r * len(act)
    # the adapter columns are padded to a whole 128-column K-tile pair (zeros in W' and in X'), so the widened GEMM
    # runs on the hand-written HIP kernels (K' % 128 == 0); the pad costs 128 / K of the base GEMM's FLOPs
    Rp = -(-R // 128) * 128 if K % 128 == 0 else R
    wide = torch.zeros(n, K + Rp, device=w.device, dtype=w.dtype)
    wide[:, :K].copy_(w)
    setattr(owner, wname, nn.Parameter(wide[:, :K], requires_grad=False))
    offs = [sum(fl.out_splits[:i]) for i in range(len(fl.out_splits))]
    fl.wide = wide
    fl.wide_meta = [(offs[i], fl.out_splits[i], j * fl.r) for j, i in enumerate(act)]


def lora_state_dict(model) -> Dict[str, torch.Tensor]:
    """PEFT-style adapter keys: base_model.model.model.layers.{i}.self_attn.q_proj.lora_A.weight ..."""
    sd = {}
    for i, layer in enumerate(model.model.layers):
        for owner, mod_name, key in ((layer.self_attn, "self_attn", "qkv"), (layer.self_attn, "self_attn", "o"),
                                     (layer.mlp, "mlp", "gate_up"), (layer.mlp, "mlp", "down")):
            if owner.lora is None:
                continue
            fl = owner.lora[key]
            for name, a, b, act in zip(fl.names, fl.A, fl.B, fl.active):
                if act:
                    pre = f"base_model.model.model.layers.{i}.{mod_name}.{name}"
                    sd[pre + ".lora_A.weight"] = a.detach()
                    sd[pre + ".lora_B.weight"] = b.detach()
    return sd


@torch.no_grad()
def merge_lora(model):
    """Fold adapters into the base weights and drop them (for export / inference)."""
    for layer in model.model.layers:
        if layer.self_attn.lora is not None:
            layer.self_attn.qkv_proj.add_(layer.self_attn.lora["qkv"].delta_weight().to(layer.self_attn.qkv_proj.dtype))
            layer.self_attn.o_proj.add_(layer.self_attn.lora["o"].delta_weight().to(layer.self_attn.o_proj.dtype))
            layer.self_attn.lora = None
        if layer.mlp.lora is not None:
            layer.mlp.gate_up_proj.add_(layer.mlp.lora["gate_up"].delta_weight().to(layer.mlp.gate_up_proj.dtype))
            layer.mlp.down_proj.add_(layer.mlp.lora["down"].delta_weight().to(layer.mlp.down_proj.dtype))
            layer.mlp.lora = None
    return model
