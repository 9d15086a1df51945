#!/usr/bin/env python3
"""Per-kernel hardware-counter summary of a training step (rocprofv3 --pmc CSVs), SURVEY §5.1: MFMA utilisation,
LDS bank conflicts and HBM traffic of every kernel the step runs.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmcA -o run -- python bench.py --steps 2 --warmup 1
    rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmcB -o run -- python bench.py ...
    python tools/pmc_step.py /tmp/pmcA /tmp/pmcB --out profiles/x.md

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (the convention of
profiles/r2_gemm_pingpong.md); effective clock = GRBM_GUI_ACTIVE / 8 / kernel time; HBM read = FETCH_SIZE (KB).
PMC passes serialise dispatches, so the overlapped optimizer update runs alone here.
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:80]


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum
    dur = defaultdict(float)
    calls = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r.get("Kernel_Name", "?"))
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                if did not in calls[k]:
                    calls[k].add(did)
                    if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if not any(dur.values()):  # no timestamps in the counter CSV: take them from the kernel trace
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    dur[short(r.get("Kernel_Name", "?"))] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return per, dur, {k: len(v) for k, v in calls.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out")
    ap.add_argument("--raw", action="store_true", help="every collected counter per call (stall breakdowns)")
    a = ap.parse_args()
    per = defaultdict(dict)
    dur, calls = {}, {}
    for d in a.dirs:
        p, du, c = load(d)
        for k, v in p.items():
            per[k].update(v)
        for k, v in du.items():
            dur[k] = max(dur.get(k, 0.0), v)
        for k, v in c.items():
            calls[k] = max(calls.get(k, 0), v)
    rows = sorted(per, key=lambda k: -dur.get(k, 0.0))[: a.top]
    tot = sum(dur.values())
    if a.raw:
        names = sorted({n for k in rows for n in per[k]})
        lines = ["| kernel | calls | us/call | " + " | ".join(names) + " |", "|---|---:|---:|" + "---:|" * len(names)]
        for k in rows:
            n = max(calls.get(k, 1), 1)
            lines.append(f"| `{k}` | {n} | {dur.get(k, 0.0) / n:.1f} | "
                         + " | ".join(f"{per[k].get(c, 0.0) / n:.4g}" for c in names) + " |")
        txt = "\n".join(lines) + "\n"
        if a.out:
            with open(a.out, "w") as fh:
                fh.write(txt)
        print(txt)
        return
    lines = ["# Per-kernel hardware counters of the training step (rocprofv3 --pmc, serialised dispatches)", "",
             f"sources: {', '.join('`' + d + '`' for d in a.dirs)}; kernel time in the PMC passes {tot / 1e3:.1f} ms", "",
             "| kernel | calls | time us | MFMA busy % | eff. clock GHz | LDS bank-conflict % | HBM read GB | read TB/s |",
             "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for k in rows:
        c = per[k]
        t = dur.get(k, 0.0)
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        mf = 100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024) if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None
        clk = g / 8 / (t * 1e3) if g and t else None  # cycles per ns
        lds = (100.0 * c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
               if c.get("SQ_LDS_IDX_ACTIVE") else None)
        rd = c["FETCH_SIZE"] * 1024 / 1e9 if "FETCH_SIZE" in c else None
        bw = rd / (t * 1e-6) / 1e3 if rd is not None and t else None

        def f(x, p=1):
            return "" if x is None else f"{x:.{p}f}"
        lines.append(f"| `{k}` | {calls.get(k, 0)} | {t:.0f} | {f(mf)} | {f(clk, 2)} | {f(lds)} | {f(rd, 2)} | {f(bw, 2)} |")
    txt = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
