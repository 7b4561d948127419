#!/usr/bin/env python3
"""Per-stream view of one steady-state training step from a rocprofv3 --kernel-trace CSV:
busy time per stream, forward / backward split of the main stream (softmax_xent marks the
boundary) and the main-stream idle gaps (time the critical path waits on other streams).

usage: step_streams.py <kernel_trace.csv>
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
# a step may update in two launches (backward(defer_tail)): the step ends at the LAST of
# a group of optimizer launches a few kernels apart
idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
print(f"step wall {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
by = collections.defaultdict(list)
for r in step:
    by[r["Stream_Id"]].append(r)
main = max(by, key=lambda s: len(by[s]))
for s, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
    print(f"stream {s:>3}: {len(rs):4d} kernels, busy {busy / 1e3:8.1f} us{'  (main)' if s == main else ''}")
ms = by[main]
sx = [i for i, r in enumerate(ms) if "softmax_xent" in r["Kernel_Name"]]
if sx:
    fwd_end = int(ms[sx[0]]["End_Timestamp"])
    print(f"forward (step start -> softmax end): {(fwd_end - t0) / 1e3:.1f} us; backward+update: {(t1 - fwd_end) / 1e3:.1f} us")
gaps = []
for p, q in zip(ms, ms[1:]):
    g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
    if g > 0:
        gaps.append((g, p["Kernel_Name"].split("(")[0][-60:], q["Kernel_Name"].split("(")[0][-60:]))
print(f"main-stream gaps: total {sum(g for g, _, _ in gaps) / 1e3:.1f} us over {len(gaps)} gaps")
for g, p, q in sorted(gaps, reverse=True)[:12]:
    print(f"  {g / 1e3:7.1f} us  after {p}  before {q}")


# Overlap accounting: a main-stream gap is only idle GPU time when no other stream runs either.
def _union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _covered(a, b, iv):
    return sum(max(0, min(b, y) - max(a, x)) for x, y in iv)


others = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for s, rs in by.items() if s != main
                 for r in rs])
main_iv = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ms])
all_iv = _union(main_iv + others)
gap_cov = sum(_covered(int(p["End_Timestamp"]), int(q["Start_Timestamp"]), others)
              for p, q in zip(ms, ms[1:]) if int(q["Start_Timestamp"]) > int(p["End_Timestamp"]))
both = sum(_covered(a, b, others) for a, b in main_iv)
idle = (t1 - t0) - sum(b - a for a, b in all_iv)
print(f"main-stream gaps covered by other streams' kernels: {gap_cov / 1e3:.1f} us "
      f"(truly idle GPU inside the step: {idle / 1e3:.1f} us)")
print(f"main and other streams running concurrently: {both / 1e3:.1f} us "
      f"({both / max(1, sum(b - a for a, b in others)):.0%} of the other streams' busy time)")
# the step's tail: the last kernels of both streams (start / end relative to the step end)
print("tail (us before step end):")
for r in step[-14:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  stream {r['Stream_Id']:>3} {(s - t1) / 1e3:8.1f} .. {(e - t1) / 1e3:8.1f}  {r['Kernel_Name'][:90]}")
