#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs: calls, mean counter value per call (FETCH_SIZE /
WRITE_SIZE are in KB).  Usage: python tools/pmc_summary.py <counter_collection.csv> [...] [--top N]"""
import csv
import sys
from collections import defaultdict


def summarize(paths, top=12):
    agg = defaultdict(lambda: [0, 0.0])
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = (r["Counter_Name"], r["Kernel_Name"][:100])
            agg[k][0] += 1
            agg[k][1] += float(r["Counter_Value"])
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]
    return [{"counter": c, "kernel": k, "calls": n, "mean_per_call": round(v / n, 1)} for (c, k), (n, v) in rows]


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    args = [a for a in args if not a.isdigit()]
    import json
    for row in summarize(args, top):
        print(json.dumps(row))
