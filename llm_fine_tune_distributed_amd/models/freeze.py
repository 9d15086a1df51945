"""Freeze policies (reference C4/F1, ``training.py:113-145``).

* ``last_n_layers`` (reference default, n=2): everything frozen except the last n decoder
  layers and the output head. SmolLM3 ties lm_head to embed_tokens, so the embedding is
  trainable too: 418,914,304 / 3,075,098,624 params = 13.62%.
* ``full``: all parameters trainable (BASELINE.json full-param SFT).
* ``lora``: base frozen, adapters trainable (see ``lora.py``).
"""
from __future__ import annotations

from typing import Tuple


def apply_freeze_policy(model, policy: str = "full", n_last: int = 2, lora_config=None) -> Tuple[int, int]:
    policy = (policy or "full").lower()
    if policy == "lora":
        from .lora import apply_lora
        apply_lora(model, lora_config)
    elif policy == "full":
        for p in model.parameters():
            p.requires_grad_(True)
    elif policy in ("last_n_layers", "reference", "last2"):
        try:
            for p in model.parameters():
                p.requires_grad_(False)
            layers = model.model.layers
            for p in layers[-n_last:].parameters():
                p.requires_grad_(True)
            model.lm_head_weight.requires_grad_(True)
        except Exception:  # reference falls back to all-trainable on any error (training.py:143-145)
            for p in model.parameters():
                p.requires_grad_(True)
    else:
        raise ValueError(f"unknown freeze policy {policy!r}")
    trainable = model.num_parameters(trainable_only=True)
    total = model.num_parameters()
    return trainable, total
