#!/usr/bin/env python3
"""GPU idle-gap analysis of a rocprofv3 kernel trace (.db): where the device waits for the host.

Merges every kernel interval (all streams) into busy spans over the LAST ``--window-ms`` of the trace (the
timed steps of a bench.py run), then reports busy / idle totals, a gap-size histogram and the largest gaps with
the kernels on either side, so launch-bound stretches of a training step (Python / autograd / hook overhead
between short kernels) show up by name.

    python tools/prof_timeline.py gpurun_out/prof/run_results.db --window-ms 600 [--out profiles/x.md]
"""
import argparse
import os
import re
import sqlite3
from collections import Counter


def load(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    return [(re.sub(r"\(.*", "", n).replace("void ", "")[:90], s, e) for n, s, e in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--window-ms", type=float, default=0.0, help="analyse only the last W ms of the trace (0 = all)")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--out")
    a = ap.parse_args()
    ks = load(a.path)
    t_end = max(e for _, _, e in ks)
    t0 = t_end - a.window_ms * 1e6 if a.window_ms else min(s for _, s, _ in ks)
    ks = [k for k in ks if k[2] > t0]
    busy = 0
    gaps = []  # (gap_ns, prev_kernel, next_kernel, at_ns)
    cur_s, cur_e, cur_last = None, None, None
    for n, s, e in ks:
        s = max(s, t0)
        if cur_e is None:
            cur_s, cur_e, cur_last = s, e, n
            continue
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_last, n, cur_e - t0))
            cur_s, cur_e, cur_last = s, e, n
        elif e > cur_e:
            cur_e, cur_last = e, n
    busy += cur_e - cur_s
    span = t_end - t0
    idle = span - busy
    hist = Counter()
    edges = [1e3, 5e3, 2e4, 1e5, 1e6, float("inf")]
    labels = ["<1 us", "1-5 us", "5-20 us", "20-100 us", "0.1-1 ms", ">1 ms"]
    hsum = Counter()
    for g, *_ in gaps:
        for ed, lb in zip(edges, labels):
            if g < ed:
                hist[lb] += 1
                hsum[lb] += g
                break
    lines = ["# GPU timeline: busy vs idle", "", f"source: `{a.path}`, window {span/1e6:.2f} ms, {len(ks)} kernels", "",
             f"busy (union of kernel intervals, all streams) {busy/1e6:.2f} ms = {100*busy/span:.1f} %; "
             f"idle {idle/1e6:.2f} ms in {len(gaps)} gaps", "", "| gap size | count | total ms |", "|---|---:|---:|"]
    for lb in labels:
        lines.append(f"| {lb} | {hist[lb]} | {hsum[lb]/1e6:.3f} |")
    lines += ["", f"## {a.top} largest gaps", "", "| gap us | at ms | after | before |", "|---:|---:|---|---|"]
    for g, p, nx, at in sorted(gaps, reverse=True)[: a.top]:
        lines.append(f"| {g/1e3:.1f} | {at/1e6:.2f} | `{p}` | `{nx}` |")
    # which kernel pairs account for the most idle time overall
    pair = Counter()
    for g, p, nx, _ in gaps:
        pair[(p, nx)] += g
    lines += ["", "## idle time by (after, before) kernel pair", "", "| total us | after | before |", "|---:|---|---|"]
    for (p, nx), g in pair.most_common(a.top):
        lines.append(f"| {g/1e3:.1f} | `{p}` | `{nx}` |")
    txt = "\n".join(lines) + "\n"
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
