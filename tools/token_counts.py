#!/usr/bin/env python3
"""Token counts of the reference's parquet rows through the chat-template paths (D3 parity report).

    python tools/token_counts.py [/root/reference/data/qa_dataset.parquet] [--template tests/fixtures/...jinja]

The offline tokenizer is the synthetic byte-level BPE (the SmolLM3 vocabulary is not available offline), so
absolute counts are unpinned against the hub tokenizer; the two template paths must agree exactly.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from llm_fine_tune_distributed_amd.data.dataset import load_qa_parquet  # noqa: E402
from llm_fine_tune_distributed_amd.data.prompts import format_prompt  # noqa: E402
from llm_fine_tune_distributed_amd.data.tokenizer import load_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("parquet", nargs="?", default="/root/reference/data/qa_dataset.parquet")
    ap.add_argument("--template", default=os.path.join(os.path.dirname(__file__), "..", "tests", "fixtures",
                                                       "smollm3_like_chat_template.jinja"))
    a = ap.parse_args()
    rows = load_qa_parquet(a.parquet)
    tk = load_tokenizer(corpus=[r["full-question"] for r in rows] + [r["answer"] for r in rows])
    msgs = [format_prompt(r)["messages"] for r in rows]
    builtin = np.array([len(tk.apply_chat_template(m)) for m in msgs])
    tk.chat_template = open(a.template).read()
    jinja = np.array([len(tk.apply_chat_template(m)) for m in msgs])
    chars = np.array([len(tk.apply_chat_template(m, tokenize=False)) for m in msgs])
    print(f"rows: {len(rows)}  (tokenizer: synthetic BPE, vocab {tk.vocab_size})")
    print(f"paths agree on every row: {bool((builtin == jinja).all())}")
    for name, v in (("rendered chars", chars), ("tokens", builtin)):
        print(f"{name:>15}: min {v.min()}  mean {v.mean():.1f}  p50 {int(np.median(v))}  p99 {int(np.percentile(v, 99))}"
              f"  max {v.max()}")
    print(f"chars/token: {chars.sum() / builtin.sum():.2f}; rows > 1024 tokens (truncated): {(builtin > 1024).sum()}")


if __name__ == "__main__":
    main()
