#!/usr/bin/env python3
"""Averages rocprofv3 --pmc counter values per kernel (name filter) over a
run's launches, skipping the first `--skip` launches of that kernel.
    python scripts/summarize_counters.py gpurun_out/sq_k4a/run_counter_collection.csv jacobi3d_tbr [--skip 2]"""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("kernel")
ap.add_argument("--skip", type=int, default=0)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.csv)) if a.kernel in r["Kernel_Name"]]
by = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in rows:
    d = r.get("Dispatch_Id") or r.get("Correlation_Id")
    by[int(d)][r["Counter_Name"]] += float(r["Counter_Value"])
    names[int(d)] = r["Kernel_Name"]
ids = sorted(by)[a.skip:]
tot = collections.defaultdict(float)
for d in ids:
    for k, v in by[d].items():
        tot[k] += v
out = {k: v / max(len(ids), 1) for k, v in sorted(tot.items())}
print(json.dumps({"kernel": names[ids[0]] if ids else None, "launches": len(ids), "avg": out}, indent=1))
