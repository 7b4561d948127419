#!/usr/bin/env python3
"""Truly idle intervals (no kernel on any stream) inside the last complete step of a kernel
trace, with the kernels on either side -- what a cross-queue wait or a host stall leaves.
usage: idle_intervals.py <kernel_trace.csv> [top]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
step = rows[idx[-2] + 1:idx[-1] + 1]


def nm(n):
    m = re.search(r"drn::(\w+)(<[^(]*)?", n)
    return ((m.group(1) + (m.group(2) or "")) if m else n[:40])[:70]


iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in step)
cur_end, last, idle = iv[0][1], iv[0][2], []
for s, e, r in iv[1:]:
    if s > cur_end:
        idle.append((s - cur_end, last, r))
    if e > cur_end:
        cur_end, last = e, r
print(f"truly idle {sum(d for d, _, _ in idle) / 1e3:.1f} us over {len(idle)} intervals")
for d, a, b in sorted(idle, key=lambda x: -x[0])[:top]:
    print(f"{d / 1e3:7.1f} us after {nm(a['Kernel_Name'])} [s{a['Stream_Id']}] before {nm(b['Kernel_Name'])} "
          f"[s{b['Stream_Id']}]")
