"""Model configuration for the decoder-only LMs this framework trains.

The reference loads ``HuggingFaceTB/SmolLM3-3B`` from the Hub (``training.py:54,97-102``).
There is no network here, so models are built from a config (HF ``config.json`` keys are
accepted) and either random-initialised or loaded from local safetensors.

SmolLM3 facts: GQA 16q/4kv, head_dim 128, 36 layers, SwiGLU 11008,
vocab 128256, tied embeddings, NoPE on every 4th layer (``no_rope_layers``), eps 1e-6.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class ModelConfig:
    model_type: str = "smollm3"
    vocab_size: int = 128256
    hidden_size: int = 2048
    intermediate_size: int = 11008
    num_hidden_layers: int = 36
    num_attention_heads: int = 16
    num_key_value_heads: int = 4
    head_dim: Optional[int] = None
    rms_norm_eps: float = 1e-6
    rope_theta: float = 2_000_000.0
    rope_scaling: Optional[Dict[str, Any]] = None
    max_position_embeddings: int = 32768
    tie_word_embeddings: bool = True
    # 1 = layer uses RoPE, 0 = NoPE layer (SmolLM3 convention).
    no_rope_layers: Optional[List[int]] = None
    no_rope_layer_interval: int = 4
    initializer_range: float = 0.02
    bos_token_id: Optional[int] = 128000
    eos_token_id: Optional[int] = 128001
    pad_token_id: Optional[int] = 128004
    torch_dtype: str = "bfloat16"
    extra: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads
        if self.no_rope_layers is None:
            if self.model_type == "smollm3":
                iv = self.no_rope_layer_interval
                self.no_rope_layers = [int((i + 1) % iv != 0) for i in range(self.num_hidden_layers)]
            else:
                self.no_rope_layers = [1] * self.num_hidden_layers
        assert len(self.no_rope_layers) >= self.num_hidden_layers
        assert self.num_attention_heads % self.num_key_value_heads == 0

    # ------------------------------------------------------------------ helpers
    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    def uses_rope(self, layer_idx: int) -> bool:
        return bool(self.no_rope_layers[layer_idx])

    def num_parameters(self) -> int:
        h, i, v = self.hidden_size, self.intermediate_size, self.vocab_size
        per_layer = h * self.qkv_size + self.q_size * h + 3 * h * i + 2 * h
        emb = v * h
        head = 0 if self.tie_word_embeddings else v * h
        return self.num_hidden_layers * per_layer + emb + head + h

    def flops_per_token(self, seq_len: int, training: bool = True, recompute: bool = False) -> float:
        """Analytic matmul FLOPs per token. Attention counted causal."""
        h = self.hidden_size
        dense = self.num_hidden_layers * (h * self.qkv_size + self.q_size * h + 3 * h * self.intermediate_size)
        dense += self.vocab_size * h
        fwd = 2.0 * dense
        # causal attention: QK^T and PV, each 2*T*d per head per token, halved by the mask
        fwd += self.num_hidden_layers * 2.0 * 2.0 * self.num_attention_heads * self.head_dim * seq_len / 2.0
        if not training:
            return fwd
        mult = 4.0 if recompute else 3.0
        return fwd * mult

    # ------------------------------------------------------------------ (de)serialisation
    def to_hf_dict(self) -> Dict[str, Any]:
        arch = {"smollm3": "SmolLM3ForCausalLM", "llama": "LlamaForCausalLM"}.get(self.model_type, "LlamaForCausalLM")
        d = {
            "architectures": [arch],
            "model_type": self.model_type,
            "vocab_size": self.vocab_size,
            "hidden_size": self.hidden_size,
            "intermediate_size": self.intermediate_size,
            "num_hidden_layers": self.num_hidden_layers,
            "num_attention_heads": self.num_attention_heads,
            "num_key_value_heads": self.num_key_value_heads,
            "head_dim": self.head_dim,
            "rms_norm_eps": self.rms_norm_eps,
            "rope_theta": self.rope_theta,
            "rope_scaling": self.rope_scaling,
            "max_position_embeddings": self.max_position_embeddings,
            "tie_word_embeddings": self.tie_word_embeddings,
            "hidden_act": "silu",
            "attention_bias": False,
            "mlp_bias": False,
            "initializer_range": self.initializer_range,
            "bos_token_id": self.bos_token_id,
            "eos_token_id": self.eos_token_id,
            "pad_token_id": self.pad_token_id,
            "torch_dtype": self.torch_dtype,
        }
        if self.model_type == "smollm3":
            d["no_rope_layers"] = list(self.no_rope_layers[: self.num_hidden_layers])
            d["no_rope_layer_interval"] = self.no_rope_layer_interval
        d.update(self.extra)
        return d

    @classmethod
    def from_hf_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in names and k != "extra"}
        # transformers>=5 moves rope params into rope_parameters
        rp = d.get("rope_parameters")
        if isinstance(rp, dict):
            if "rope_theta" in rp:
                kw["rope_theta"] = rp["rope_theta"]
            if rp.get("rope_type", "default") not in ("default", None):
                kw["rope_scaling"] = rp
        if isinstance(kw.get("eos_token_id"), list):
            kw["eos_token_id"] = kw["eos_token_id"][0]
        kw.setdefault("model_type", d.get("model_type", "llama"))
        if kw["model_type"] not in ("smollm3", "llama"):
            kw["model_type"] = "llama"
        return cls(**kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "ModelConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_hf_dict(json.load(f))

    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(self.to_hf_dict(), f, indent=2)


# ---------------------------------------------------------------------------- presets
def smollm3_3b() -> ModelConfig:
    """HuggingFaceTB/SmolLM3-3B (reference model, ``training.py:54``)."""
    return ModelConfig(model_type="smollm3")


def llama3_8b() -> ModelConfig:
    """Meta-Llama-3-8B shape (BASELINE.json config #5)."""
    return ModelConfig(
        model_type="llama", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
        num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0,
        max_position_embeddings=8192, tie_word_embeddings=False, rms_norm_eps=1e-5,
        eos_token_id=128001, pad_token_id=None,
    )


def tiny(model_type: str = "smollm3", **kw) -> ModelConfig:
    """Small config with the same structure (GQA, NoPE interval, tied head) for tests."""
    base = dict(
        model_type=model_type, vocab_size=1024, hidden_size=128, intermediate_size=256,
        num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, head_dim=32,
        rope_theta=10000.0, max_position_embeddings=1024, tie_word_embeddings=(model_type == "smollm3"),
        bos_token_id=1, eos_token_id=2, pad_token_id=2,
    )
    base.update(kw)
    return ModelConfig(**base)


PRESETS = {
    "smollm3-3b": smollm3_3b,
    "HuggingFaceTB/SmolLM3-3B": smollm3_3b,
    "llama3-8b": llama3_8b,
    "meta-llama/Meta-Llama-3-8B": llama3_8b,
    "tiny": tiny,
    "tiny-llama": lambda: tiny("llama"),
    # tiny depth/width with the real head_dim (128) the HIP attention kernels are built for (GPU tests)
    "tiny-gpu": lambda: tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                             intermediate_size=512, vocab_size=1024, num_hidden_layers=3),
}


def get_config(name_or_path: str) -> ModelConfig:
    if name_or_path in PRESETS:
        return PRESETS[name_or_path]()
    if os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        return ModelConfig.from_pretrained(name_or_path)
    raise ValueError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
