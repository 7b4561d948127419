#!/usr/bin/env python3
"""Per-dispatch roofline of the last training step in scripts/pmc_step.sh's passes: for every
convolution launch its time, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE), MFMA FLOPs
(SQ_INSTS_MFMA x 16x16x32x2) and the time a kernel at the achievable rates would take
(max(bytes / BW, flops / PEAK)); grouped by kernel configuration, sorted by the time lost
against that bound -- where the convolution time goes.

usage: pmc_dispatch.py <outdir> [BW_TBps=5.5] [PEAK_TFLOPs=2000]
"""
import collections
import csv
import glob
import os
import sys


def step_rows(pass_dir):
    f = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    by = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        e = by.setdefault(d, {"name": r["Kernel_Name"], "t0": int(r["Start_Timestamp"]),
                              "t1": int(r["End_Timestamp"]), "grid": int(r["Grid_Size"]),
                              "wg": int(r["Workgroup_Size"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = [by[d] for d in sorted(by)]
    idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["name"]]
    idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
    return rows[idx[-2] + 1: idx[-1] + 1]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("drn::", "")


def main():
    out = sys.argv[1]
    bw = float(sys.argv[2]) * 1e12 if len(sys.argv) > 2 else 5.5e12
    peak = float(sys.argv[3]) * 1e12 if len(sys.argv) > 3 else 2.0e15
    p0, p1, p2 = (step_rows(os.path.join(out, f"p{i}")) for i in range(3))
    n = min(len(p0), len(p1), len(p2))
    groups = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
    tot = [0.0, 0.0]
    for a, b, c in zip(p0[:n], p1[:n], p2[:n]):
        nm = short(b["name"])
        if short(a["name"]) != nm or short(c["name"]) != nm:
            raise SystemExit(f"passes disagree on the dispatch order: {nm}")
        us = (b["t1"] - b["t0"]) / 1e3
        byt = (2 * b.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
        fl = a.get("SQ_INSTS_MFMA", 0) * 16 * 16 * 32 * 2
        ideal = max(byt / bw, fl / peak) * 1e6
        g = groups[nm]
        g[0] += 1
        g[1] += us
        g[2] += ideal
        g[3] += byt
        g[4] += fl
        tot[0] += us
        tot[1] += ideal
    print(f"# last step: {n} dispatches, {tot[0]:.0f} us kernel time, {tot[1]:.0f} us at "
          f"max(bytes / {bw / 1e12:.1f} TB/s, flops / {peak / 1e12:.0f} TF/s)")
    print(f"{'kernel configuration':86s} {'n':>3s} {'us':>7s} {'bound us':>8s} {'lost us':>7s} {'GB/s':>6s} {'TF/s':>6s}")
    for nm, (k, us, ideal, byt, fl) in sorted(groups.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
        if us - ideal < 5:
            continue
        print(f"{nm[:86]:86s} {k:3d} {us:7.0f} {ideal:8.0f} {us - ideal:7.0f} {byt / us / 1e3:6.0f} {fl / us / 1e6:6.0f}")


if __name__ == "__main__":
    main()
