#!/usr/bin/env python3
"""Summarise one steady-state training step from a rocprofv3 --kernel-trace CSV.

usage: prof_step.py <kernel_trace.csv> [min_us]
Splits the trace at the fused SGD kernel (one per step) and prints per-dispatch durations of
the last complete step plus a per-kernel-family total.
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
# a step may update in two launches (backward(defer_tail)): the step ends at the LAST of
# a group of optimizer launches a few kernels apart
idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"kernels/step {len(step)}  wall {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms")
fam = collections.defaultdict(float)
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("drn::", "")
    fam[n] += d
    if d > thr:
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        print(f"{d:9.1f}us wg={g:>6}x{r['Grid_Size_Y']:>3} vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']:>6} {n}")
print("--- per family (us/step) ---")
for n, d in sorted(fam.items(), key=lambda x: -x[1]):
    print(f"{d:10.1f}  {n}")
