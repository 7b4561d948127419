#!/usr/bin/env python3
"""Which hardware queue every HIP stream of a profiled run landed on (rocprofv3 kernel trace).

usage: queue_map.py <kernel_trace.csv> [label]
With GPU_MAX_HW_QUEUES=4 (the default on these boxes) a process maps its streams onto at most 4
hardware queues; two streams sharing a queue serialize (round 3 measured 12.9 vs 11.3 ms when the
high-priority main stream shared one with the side stream). For each (Stream_Id, Queue_Id) pair:
dispatches, busy time and the most frequent kernels, so a data-parallel run records where the
critical-path stream, the weight-gradient side stream, the report stream's collectives (RCCL)
and the P2P comm stream execute.
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    by = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    for r in rows:
        k = (r.get("Stream_Id", "?"), r.get("Queue_Id", "?"))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        e = by[k]
        e[0] += 1
        e[1] += d
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("drn::", "")
        e[2][name.split("<")[0][:40]] += 1
    queues = collections.defaultdict(set)
    for s, q in by:
        queues[q].add(s)
    print(f"# stream -> hardware queue map {label} ({len(rows)} dispatches, {len(queues)} queues)")
    print(f"{'stream':>7} {'queue':>6} {'kernels':>8} {'busy ms':>9}  top kernels")
    for (s, q), (n, busy, names) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        top = ", ".join(f"{k} x{v}" for k, v in names.most_common(3))
        print(f"{s:>7} {q:>6} {n:8d} {busy / 1e3:9.2f}  {top}")
    shared = {q: sorted(ss) for q, ss in queues.items() if len(ss) > 1}
    print(f"# queues shared by several streams: {shared if shared else 'none'}")


if __name__ == "__main__":
    main()
