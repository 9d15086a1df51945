"""Dataset loading, split and tokenisation (reference D0-D3, ``training.py:155-212``).

* ``load_qa_parquet``: the reference's ``load_dataset("parquet", ...)["train"]`` (pyarrow).
* ``train_test_split``: same permutation as ``datasets.Dataset.train_test_split(test_size,
  seed)`` (``np.random.default_rng(seed).permutation``; test = first ceil(test_size*n)), so a
  given seed picks the same 2,560/285 rows as the reference.
* ``TokenizedDataset``: chat-template rendering + tokenisation of every row, stored as one flat
  int32 token array + int64 offsets (CSR). The native collator (csrc/data_pipeline.cpp) builds
  micro-batches straight from this layout. Loss is over all tokens like the reference (TRL
  without assistant-only masking); ``assistant_only_loss`` masks the prompt instead.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .prompts import format_prompt


def load_qa_parquet(path: str) -> List[Dict[str, str]]:
    import pyarrow.parquet as pq
    tbl = pq.read_table(path)
    return tbl.to_pylist()


def load_jsonl(path: str) -> List[Dict]:
    import json
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


def train_test_split(rows: Sequence, test_size: float = 0.1, seed: int = 42):
    n = len(rows)
    n_test = math.ceil(test_size * n) if isinstance(test_size, float) else int(test_size)
    n_train = n - n_test
    perm = np.random.default_rng(seed).permutation(n)
    test_idx, train_idx = perm[:n_test], perm[n_test:n_test + n_train]
    return [rows[i] for i in train_idx], [rows[i] for i in test_idx]


class TokenizedDataset:
    """CSR token storage: ``tokens`` int32 [N_tokens], ``offsets`` int64 [n+1], optional
    ``loss_start`` int32 [n] (first token that contributes to the loss)."""

    def __init__(self, tokens: torch.Tensor, offsets: torch.Tensor, loss_start: Optional[torch.Tensor] = None):
        self.tokens = tokens.to(torch.int32).contiguous()
        self.offsets = offsets.to(torch.int64).contiguous()
        self.loss_start = loss_start

    def __len__(self):
        return self.offsets.numel() - 1

    def lengths(self) -> torch.Tensor:
        return self.offsets[1:] - self.offsets[:-1]

    def __getitem__(self, i) -> List[int]:
        return self.tokens[self.offsets[i]:self.offsets[i + 1]].tolist()

    @classmethod
    def from_token_lists(cls, seqs: Iterable[List[int]], loss_start: Optional[List[int]] = None):
        seqs = list(seqs)
        lens = torch.tensor([len(s) for s in seqs], dtype=torch.int64)
        off = torch.zeros(len(seqs) + 1, dtype=torch.int64)
        off[1:] = lens.cumsum(0)
        flat = torch.tensor([t for s in seqs for t in s], dtype=torch.int32)
        ls = torch.tensor(loss_start, dtype=torch.int32) if loss_start is not None else None
        return cls(flat, off, ls)

    @classmethod
    def synthetic(cls, n: int, vocab_size: int, min_len: int, max_len: int, seed: int = 0):
        """Random-token samples with lengths uniform in [min_len, max_len] (benchmarks)."""
        g = torch.Generator().manual_seed(seed)
        lens = torch.randint(min_len, max_len + 1, (n,), generator=g)
        off = torch.zeros(n + 1, dtype=torch.int64)
        off[1:] = lens.cumsum(0)
        toks = torch.randint(0, vocab_size, (int(off[-1]),), generator=g, dtype=torch.int32)
        return cls(toks, off)


def to_messages(row: Dict) -> List[Dict[str, str]]:
    if "messages" in row:
        return row["messages"]
    if "full-question" in row:
        return format_prompt(row)["messages"]
    if "question" in row and "answer" in row:
        q = f"For {row['topic']}, {row['question']}" if "topic" in row else row["question"]
        return format_prompt({"full-question": q, "answer": row["answer"]})["messages"]
    raise KeyError("row needs 'messages' or ('full-question', 'answer')")


def tokenize_rows(rows: Sequence[Dict], tokenizer, max_length: Optional[int] = None,
                  assistant_only_loss: bool = False, text_field: str = "text") -> TokenizedDataset:
    texts, starts = [], []
    for r in rows:
        if text_field in r and "messages" not in r and "full-question" not in r:
            texts.append(r[text_field])
            starts.append(0)
            continue
        msgs = to_messages(r)
        full = tokenizer.apply_chat_template(msgs, tokenize=False)
        texts.append(full)
        if assistant_only_loss:
            prompt = tokenizer.apply_chat_template([m for m in msgs if m["role"] != "assistant"], tokenize=False,
                                                   add_generation_prompt=True)
            starts.append(len(tokenizer.encode(prompt)))
        else:
            starts.append(0)
    ids = tokenizer.encode_batch(texts) if hasattr(tokenizer, "encode_batch") else [tokenizer.encode(t) for t in texts]
    if max_length:
        ids = [s[:max_length] for s in ids]  # TRL truncation at max_length (training.py:282)
    return TokenizedDataset.from_token_lists(ids, starts if assistant_only_loss else None)


def _fingerprint(rows: Sequence[Dict], tokenizer, **kw) -> str:
    import hashlib
    import json
    h = hashlib.sha256()
    h.update(json.dumps(kw, sort_keys=True, default=str).encode())
    tk = getattr(tokenizer, "_tk", None)
    h.update((tk.to_str() if tk is not None else repr(type(tokenizer))).encode())
    h.update(str(getattr(tokenizer, "chat_template", None)).encode())
    for r in rows:
        h.update(json.dumps(r, sort_keys=True, default=str).encode())
    return h.hexdigest()[:24]


def cached_tokenize(rows: Sequence[Dict], tokenizer, cache_dir: Optional[str], is_main: bool = True,
                    barrier: Optional[Callable[[], None]] = None, max_length: Optional[int] = None,
                    assistant_only_loss: bool = False, text_field: str = "text") -> TokenizedDataset:
    """TRL's ``main_process_first`` tokenisation: rank 0 renders + tokenises and writes the
    CSR arrays to ``cache_dir/tokenized-<fingerprint>.pt``; the other ranks wait at ``barrier`` and load
    them. The fingerprint covers the rows, the tokenizer (vocabulary + template) and the options, so a
    rerun with the same inputs loads instead of re-tokenising. Without ``cache_dir`` every rank tokenises."""
    import os
    kw = dict(max_length=max_length, assistant_only_loss=assistant_only_loss, text_field=text_field)
    if not cache_dir:
        return tokenize_rows(rows, tokenizer, **kw)
    path = os.path.join(cache_dir, f"tokenized-{_fingerprint(rows, tokenizer, **kw)}.pt")

    def load():
        d = torch.load(path, weights_only=True)
        return TokenizedDataset(d["tokens"], d["offsets"], d.get("loss_start"))

    ds = None
    if is_main:
        if os.path.exists(path):
            ds = load()
        else:
            ds = tokenize_rows(rows, tokenizer, **kw)
            os.makedirs(cache_dir, exist_ok=True)
            tmp = f"{path}.tmp{os.getpid()}"
            torch.save({"tokens": ds.tokens, "offsets": ds.offsets, "loss_start": ds.loss_start}, tmp)
            os.replace(tmp, path)
    if barrier is not None:
        barrier()
    if ds is None:
        ds = load() if os.path.exists(path) else tokenize_rows(rows, tokenizer, **kw)  # no shared filesystem
    return ds
