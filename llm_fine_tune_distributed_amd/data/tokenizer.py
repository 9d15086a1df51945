"""Tokenizer adapter (reference M3: ``pad_token = eos_token``, ``padding_side = "right"``,
``training.py:92-95``).

* If a directory with ``tokenizer.json`` is given (e.g. a local SmolLM3 snapshot or a saved
  ``best_model/``), the HF ``tokenizers`` (Rust) tokenizer is loaded from it.
* Otherwise (offline benchmarks) a byte-level BPE is trained on the fly on the unique texts of
  the corpus plus the system prompt. Frequent words become single tokens but whole sentences
  never do (min_frequency=2 over unique texts), so samples land near the ~4 chars/token of a
  real Llama-3 style vocabulary. Token ids stay below the model vocab (128256), so GEMM and
  cross-entropy shapes are exactly those of the real model.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, List, Optional

from . import chat_template as chat_template_mod

SPECIAL_TOKENS = ["<|begin_of_text|>", "<|end_of_text|>", "<|im_start|>", "<|im_end|>",
                  "<|finetune_right_pad_id|>", "<think>", "</think>"]


class SFTTokenizer:
    def __init__(self, tk, eos_token: str = "<|im_end|>", bos_token: Optional[str] = None,
                 pad_token: Optional[str] = None, chat_kwargs: Optional[dict] = None,
                 chat_template: Optional[str] = None):
        self._tk = tk
        self.chat_template = chat_template  # the tokenizer's own Jinja template (None: built-in renderer)
        self.eos_token = eos_token
        self.bos_token = bos_token
        self.pad_token = pad_token or eos_token  # reference: pad = eos
        self.padding_side = "right"
        self.chat_kwargs = chat_kwargs or {}

    # ------------------------------------------------------------------ ids
    def token_to_id(self, t: str) -> Optional[int]:
        return self._tk.token_to_id(t)

    @property
    def eos_token_id(self) -> int:
        return self.token_to_id(self.eos_token)

    @property
    def pad_token_id(self) -> int:
        return self.token_to_id(self.pad_token)

    @property
    def bos_token_id(self) -> Optional[int]:
        return self.token_to_id(self.bos_token) if self.bos_token else None

    @property
    def vocab_size(self) -> int:
        return self._tk.get_vocab_size()

    def __len__(self):
        return self.vocab_size

    # ------------------------------------------------------------------ text
    def encode(self, text: str) -> List[int]:
        return self._tk.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self._tk.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids: Iterable[int], skip_special_tokens: bool = False) -> str:
        return self._tk.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def __call__(self, text: str):
        return {"input_ids": self.encode(text)}

    def apply_chat_template(self, messages: List[Dict[str, str]], tokenize: bool = True,
                            add_generation_prompt: bool = False, enable_thinking: Optional[bool] = None,
                            chat_template: Optional[str] = None, **kwargs):
        """HF semantics: the tokenizer's Jinja template when it has one (extra kwargs such as
        ``enable_thinking`` reach the template), else the built-in SmolLM3-style ChatML renderer."""
        tpl = chat_template or self.chat_template
        if tpl:
            if enable_thinking is not None:
                kwargs["enable_thinking"] = enable_thinking
            text = chat_template_mod.render_jinja(
                tpl, messages, add_generation_prompt=add_generation_prompt,
                special_tokens={"bos_token": self.bos_token, "eos_token": self.eos_token,
                                "pad_token": self.pad_token}, **kwargs)
        else:
            text = chat_template_mod.render(messages, add_generation_prompt=add_generation_prompt,
                                            enable_thinking=bool(enable_thinking), **self.chat_kwargs)
        return self.encode(text) if tokenize else text

    # ------------------------------------------------------------------ io
    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        self._tk.save(os.path.join(path, "tokenizer.json"))
        with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
            cfg = {"eos_token": self.eos_token, "bos_token": self.bos_token, "pad_token": self.pad_token,
                   "padding_side": self.padding_side, "tokenizer_class": "PreTrainedTokenizerFast"}
            if self.chat_template:
                cfg["chat_template"] = self.chat_template
            else:
                cfg["chat_template_style"] = "smollm3-chatml"
            json.dump(cfg, f, indent=2)

    @classmethod
    def from_pretrained(cls, path: str) -> "SFTTokenizer":
        from tokenizers import Tokenizer
        tk = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        cfg = {}
        p = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(p):
            with open(p) as f:
                cfg = json.load(f)

        def tok(v):
            return v.get("content") if isinstance(v, dict) else v

        eos = tok(cfg.get("eos_token")) or "<|im_end|>"
        tpl = chat_template_mod.select_template(cfg.get("chat_template"))
        jp = os.path.join(path, "chat_template.jinja")  # newer transformers save the template as its own file
        if tpl is None and os.path.exists(jp):
            with open(jp) as f:
                tpl = f.read()
        return cls(tk, eos_token=eos, bos_token=tok(cfg.get("bos_token")), pad_token=tok(cfg.get("pad_token")),
                   chat_template=tpl)


def train_synthetic_tokenizer(texts: Iterable[str], vocab_size: int = 16384) -> SFTTokenizer:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, special_tokens=SPECIAL_TOKENS,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    uniq = sorted(set(texts))
    tk.train_from_iterator(uniq, trainer=tr)
    return SFTTokenizer(tk, eos_token="<|im_end|>", bos_token=None, pad_token="<|im_end|>")


def load_tokenizer(path: Optional[str] = None, corpus: Optional[Iterable[str]] = None) -> SFTTokenizer:
    if path and os.path.exists(os.path.join(path, "tokenizer.json")):
        return SFTTokenizer.from_pretrained(path)
    from .prompts import WILDERNESS_EXPERT_SYSTEM_PROMPT
    from .synthetic import generate_qa
    texts = [WILDERNESS_EXPERT_SYSTEM_PROMPT]
    if corpus is None:
        rows = generate_qa(2845, seed=42)
        texts += [r["full-question"] for r in rows] + [r["answer"] for r in rows]
    else:
        texts += list(corpus)
    return train_synthetic_tokenizer(texts)
