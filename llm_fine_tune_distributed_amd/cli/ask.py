"""Inference CLI (reference ``ask_tuned_model.py`` / ``ask_original_model.py``).

    python -m llm_fine_tune_distributed_amd.cli.ask "How do I tie a bowline?" [--model outputs/best_model]

Loads an HF-layout directory (safetensors + config + tokenizer) in bf16 on the GPU (CPU fallback),
applies the chat template with the wilderness system prompt and ``add_generation_prompt=True``,
samples with the reference's settings (T=0.6, top_p=0.95, top_k=40, repetition_penalty=1.1) and
prints the assistant span.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch


def load_model(path: str, device=None):
    from ..data.tokenizer import load_tokenizer
    from ..models import build_model, get_config
    from ..train.checkpoint import from_pretrained
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    if os.path.isdir(path):
        model = from_pretrained(path, device=device, dtype=torch.bfloat16 if device != "cpu" else torch.float32)
        tok = load_tokenizer(path)
    else:  # preset (random init) — the base hub model is not downloadable offline
        model = build_model(get_config(path), device=device, dtype=torch.bfloat16 if device != "cpu" else torch.float32)
        tok = load_tokenizer(None)
    return model, tok


def ask_question(model, tokenizer, question: str, max_new_tokens: int = 3768, enable_thinking: bool = False,
                 seed=None, **sampling) -> str:
    from ..data.chat_template import assistant_span
    from ..data.prompts import WILDERNESS_EXPERT_SYSTEM_PROMPT
    from ..inference.generation import generate
    msgs = [{"role": "system", "content": WILDERNESS_EXPERT_SYSTEM_PROMPT}, {"role": "user", "content": question}]
    prompt = tokenizer.apply_chat_template(msgs, tokenize=False, add_generation_prompt=True,
                                           enable_thinking=enable_thinking)
    ids = tokenizer.encode(prompt)
    kw = dict(temperature=0.6, top_p=0.95, top_k=40, repetition_penalty=1.1, do_sample=True)
    kw.update(sampling)
    out = generate(model, ids, max_new_tokens=max_new_tokens, eos_token_id=tokenizer.eos_token_id, seed=seed, **kw)
    return assistant_span(prompt + tokenizer.decode(out))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("question", nargs="*")
    ap.add_argument("--model", default="outputs/best_model")
    ap.add_argument("--max-new-tokens", type=int, default=3768)
    ap.add_argument("--enable-thinking", action="store_true")
    ap.add_argument("--seed", type=int, default=None)
    a = ap.parse_args(argv)
    if not a.question:
        print('Usage: python -m llm_fine_tune_distributed_amd.cli.ask "Your question here"')
        sys.exit(1)
    q = " ".join(a.question)
    print(f"Question: {q}\n")
    model, tok = load_model(a.model)
    print("Answer:")
    print(ask_question(model, tok, q, a.max_new_tokens, a.enable_thinking, seed=a.seed))


if __name__ == "__main__":
    main()
