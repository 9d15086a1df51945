"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel-name substring, the mean of every counter over
its dispatches (the first warmup dispatches of pmc_tn.py are included; they are identical work).

    python tools/pmc_csv.py <csv> [<csv> ...] --match g4_kernel,Cijk
"""
import argparse
import csv
import collections

ap = argparse.ArgumentParser()
ap.add_argument("csv", nargs="+")
ap.add_argument("--match", default="")
a = ap.parse_args()
pats = [p for p in a.match.split(",") if p]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in a.csv:
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            key = next((p for p in pats if p in name), None) if pats else name[:60]
            if key is None:
                continue
            d = (path, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            disp[key].add(d)
            vals[key][r["Counter_Name"]] += float(r["Counter_Value"])
for key, cs in vals.items():
    n = max(1, len(disp[key]))
    print(f"## {key} ({n} dispatches)")
    for c in sorted(cs):
        print(f"  {c:32s} {cs[c] / n:,.0f}")
