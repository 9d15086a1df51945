#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (.db or kernel_stats.csv) into a per-kernel table.

    python tools/prof_summary.py gpurun_out/prof2/run_results.db [--top 40] [--out profiles/x.md]
"""
import argparse
import csv
import os
import re
import sqlite3
from collections import defaultdict


def load_db(path, window=None):
    """window = (regex, skip): keep only the kernels that start after the end of the skip-th kernel whose name
    matches regex and end before the end of the last one (e.g. "adamw_kernel", 2 x warmup steps: the timed steps)."""
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    if window is not None:
        rx, skip = re.compile(window[0]), window[1]
        marks = [e for n, s, e in rows if rx.search(n)]
        if len(marks) > skip:
            lo, hi = marks[skip - 1] if skip > 0 else rows[0][1], marks[-1]
            rows = [(n, s, e) for n, s, e in rows if s >= lo and e <= hi]
    return [(n, (e - s) / 1e3) for n, s, e in rows]  # us


def load_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "")
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--window", nargs=2, metavar=("REGEX", "SKIP"),
                    help="only kernels between the end of the SKIP-th REGEX kernel and the end of the last one")
    a = ap.parse_args()
    win = (a.window[0], int(a.window[1])) if a.window else None
    rows = load_db(a.path, win) if a.path.endswith(".db") else load_csv(a.path)
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for n, us in rows:
        k = short(n)
        agg[k][0] += 1
        agg[k][1] += us
        agg[k][2] = max(agg[k][2], us)
    total = sum(v[1] for v in agg.values())
    lines = [f"# {a.title}", "", f"source: `{a.path}` — {len(rows)} dispatches, total kernel time {total/1e3:.2f} ms", "",
             "| kernel | calls | total ms | % | avg us | max us |", "|---|---:|---:|---:|---:|---:|"]
    for k, (c, t, m) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        lines.append(f"| `{k}` | {c} | {t/1e3:.2f} | {100*t/total:.1f} | {t/c:.1f} | {m:.1f} |")
    txt = "\n".join(lines) + "\n"
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
