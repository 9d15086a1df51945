"""Run status from structured artifacts (replaces the reference's kubectl monitor scripts, L4).

    python -m llm_fine_tune_distributed_amd.cli.status OUTPUT_DIR

Prints the latest logged train/eval metrics (``metrics.jsonl``), checkpoints present, and the
training summary if the run finished.
"""
from __future__ import annotations

import json
import os
import sys


def status(out_dir: str) -> dict:
    rep = {"output_dir": out_dir}
    for cand in (os.path.join(out_dir, "metrics.jsonl"), os.path.join(out_dir, "checkpoints", "metrics.jsonl")):
        if os.path.exists(cand):
            last_train = last_eval = None
            n = 0
            with open(cand) as f:
                for line in f:
                    r = json.loads(line)
                    n += 1
                    if "loss" in r:
                        last_train = r
                    if "eval_loss" in r:
                        last_eval = r
            rep.update(metrics_file=cand, log_records=n, last_train=last_train, last_eval=last_eval)
            break
    ck_dir = os.path.join(out_dir, "checkpoints") if os.path.isdir(os.path.join(out_dir, "checkpoints")) else out_dir
    rep["checkpoints"] = sorted(d for d in os.listdir(ck_dir) if d.startswith("checkpoint-")) if os.path.isdir(ck_dir) else []
    s = os.path.join(out_dir, "training_summary.json")
    if os.path.exists(s):
        with open(s) as f:
            rep["summary"] = json.load(f)
    rep["best_model"] = os.path.isdir(os.path.join(out_dir, "best_model"))
    return rep


def main(argv=None):
    argv = argv if argv is not None else sys.argv[1:]
    out = argv[0] if argv else os.getenv("OUTPUT_DIR", "/tmp/models")
    print(json.dumps(status(out), indent=2, default=str))


if __name__ == "__main__":
    main()
