#!/usr/bin/env python3
"""Sum a rocprofv3 counter_collection.csv per kernel: pmc_sum.py <csv> [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", "")[:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if sub in k:
        print(k, {a: f"{b:.4g}" for a, b in sorted(v.items())})
