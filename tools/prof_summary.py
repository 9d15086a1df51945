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


def load_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
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
    a = ap.parse_args()
    rows = load_db(a.path) if a.path.endswith(".db") else load_csv(a.path)
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
