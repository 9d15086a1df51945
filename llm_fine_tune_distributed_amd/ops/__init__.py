"""Fused ops: HIP/CDNA4 kernels (GPU) with PyTorch reference implementations (CPU/oracle)."""
from . import reference
from ._ext import load as load_extension, use_hip, hip_disabled
from .fused import (
    IGNORE_INDEX,
    add_rms_norm,
    bump_param_epoch,
    decode_attention,
    dgrad_mm,
    dropout_add,
    embedding,
    attn_out_linear,
    qkv_in_linear,
    wgrad_carry_scope,
    flash_attention,
    fuse_swiglu_down,
    linear,
    linear_rope,
    linear_swiglu,
    lm_head_cross_entropy,
    lora_inplace_ok,
    lora_linear,
    lora_qkv_rope_attention,
    lora_swiglu_mlp,
    qkv_rope_attention,
    register_param_sync,
    rms_norm,
    rope_,
    set_cu_budget,
    cu_budget,
    swiglu,
    swiglu_linear,
    swiglu_mlp,
)
from .optim_kernels import adamw_flat_, grad_norm_flat, sumsq_list

__all__ = [
    "reference", "load_extension", "use_hip", "hip_disabled", "IGNORE_INDEX", "add_rms_norm", "bump_param_epoch", "decode_attention", "dropout_add",
    "attn_out_linear", "qkv_in_linear", "wgrad_carry_scope", "embedding", "flash_attention", "linear", "linear_rope", "linear_swiglu", "lora_inplace_ok", "lora_linear", "lora_qkv_rope_attention", "lora_swiglu_mlp", "lm_head_cross_entropy", "qkv_rope_attention", "register_param_sync", "rms_norm", "rope_", "set_cu_budget", "cu_budget", "swiglu",
    "swiglu_linear", "swiglu_mlp", "dgrad_mm", "fuse_swiglu_down", "adamw_flat_", "grad_norm_flat", "sumsq_list",
]
