"""Synthetic Q&A data with the reference dataset's schema and length statistics.

The reference trains on ``data/qa_dataset.parquet`` (2,845 rows of
``{"full-question": "For {topic}, {question}", "answer"}``, SURVEY.md §2.1: question
23-116 chars, answer 1-406 chars, 6 topics). Benchmarks here must not depend on that
file (BASELINE.json: synthetic data), so this module generates rows with the same schema,
topic mix and length distribution, deterministically from a seed.
"""
from __future__ import annotations

import random
from typing import Dict, List

from .prompts import TOPICS

_SUBJECTS = ["a tarp", "the spare tire", "a bowline", "wild berries", "a small burn", "coolant", "a campfire",
             "a sprained ankle", "cups to milliliters", "baking soda", "a clove hitch", "brake fluid", "a signal mirror",
             "drinking water", "a trucker's hitch", "tire pressure", "eggs", "a splint", "miles to kilometers",
             "a shelter", "the oil level", "a figure-eight knot", "butter", "shock", "ounces to grams", "a compass"]
_VERBS = ["check", "use", "tie", "treat", "store", "replace", "substitute", "convert", "build", "purify", "inspect",
          "prepare", "identify", "measure", "secure"]
_Q = ["How do I {v} {s}?", "What is the best way to {v} {s}?", "Why should I {v} {s} regularly?",
      "When is it safe to {v} {s}?", "What tools do I need to {v} {s}?", "Can I {v} {s} without help?",
      "What mistakes should I avoid when I {v} {s}?"]
_A_SENT = ["First, {v} {s} carefully and keep your hands clear.", "Always make sure {s} is dry before you start.",
           "This matters because small errors compound quickly in the field.",
           "If you are unsure, ask an expert or consult the manual.", "Repeat the check every few days.",
           "Keep a spare on hand in case of emergency.", "Work slowly and double-check each step.",
           "Use clean materials to avoid contamination.", "Never {v} {s} near an open flame.",
           "A common substitute works in a pinch, but expect a slightly different result.",
           "Measure twice so the conversion is exact.", "Seek medical help if symptoms get worse."]


def generate_qa(n: int = 2845, seed: int = 42) -> List[Dict[str, str]]:
    """Rows ``{"full-question", "answer", "topic"}`` (topic kept for reference; not used by training)."""
    rng = random.Random(seed)
    weights = [500, 497, 493, 491, 487, 377]  # reference topic counts
    rows = []
    for _ in range(n):
        topic = rng.choices(TOPICS, weights=weights)[0]
        s, v = rng.choice(_SUBJECTS), rng.choice(_VERBS)
        q = rng.choice(_Q).format(v=v, s=s)
        n_sent = max(1, min(6, int(rng.gauss(2.2, 1.2))))
        ans = " ".join(rng.choice(_A_SENT).format(v=v, s=s) for _ in range(n_sent))[:406]
        rows.append({"full-question": f"For {topic}, {q[0].lower() + q[1:]}", "answer": ans, "topic": topic})
    return rows


def write_parquet(rows: List[Dict[str, str]], path: str) -> None:
    import pyarrow as pa
    import pyarrow.parquet as pq
    tbl = pa.table({"full-question": [r["full-question"] for r in rows], "answer": [r["answer"] for r in rows]})
    pq.write_table(tbl, path, compression="snappy")
