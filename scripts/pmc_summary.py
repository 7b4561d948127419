#!/usr/bin/env python3
"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel name (mean per dispatch)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(disp[k])
    print(f"{k}  (dispatches={n})")
    for c, v in sorted(d.items()):
        print(f"    {c:28s} {v / n:14.0f}")
