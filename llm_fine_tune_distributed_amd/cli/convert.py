"""JSONL -> Parquet conversion (reference ``convert_to_parquet.py``):
``{"topic","question","answer"}`` -> ``{"full-question": "For {topic}, {question}", "answer"}`` (snappy)."""
from __future__ import annotations

import argparse
import json
import os


def convert(input_file: str, output_file: str, verbose: bool = True):
    import pyarrow as pa
    import pyarrow.parquet as pq
    fq, ans = [], []
    with open(input_file, encoding="utf-8") as f:
        for n, line in enumerate(f, 1):
            try:
                r = json.loads(line.strip())
                fq.append(f"For {r['topic']}, {r['question']}")
                ans.append(r["answer"])
            except (json.JSONDecodeError, KeyError) as e:
                if verbose:
                    print(f"Warning: skipping invalid record on line {n}: {e}")
    pq.write_table(pa.table({"full-question": fq, "answer": ans}), output_file, compression="snappy")
    if verbose:
        a, b = os.path.getsize(input_file) / 2**20, os.path.getsize(output_file) / 2**20
        print(f"Loaded {len(fq)} records; JSONL {a:.2f} MB -> Parquet {b:.2f} MB ({(a - b) / a * 100:.1f}% smaller)")
    return len(fq)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", default="data/final_qa_data_unique.jsonl")
    ap.add_argument("--output", default="data/qa_dataset.parquet")
    a = ap.parse_args(argv)
    convert(a.input, a.output)


if __name__ == "__main__":
    main()
