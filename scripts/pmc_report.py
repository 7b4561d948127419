#!/usr/bin/env python3
"""Per-kernel-family PMC summary of the LAST training step in scripts/pmc_step.sh's passes.

usage: pmc_report.py <outdir>
Columns: dispatches, summed counters, LDS bank-conflict cycles as a share of LDS-array cycles,
MFMA-busy share of SQ busy cycles (raw counter ratio, uncalibrated), and HBM bytes from
FETCH_SIZE (x2: on gfx950 it reads half of a wide streaming read) + WRITE_SIZE (KiB units).
"""
import collections
import csv
import glob
import os
import sys


def last_step(pass_dir):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"),
                                              recursive=True)[0])))
    by_disp = collections.defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("drn::", "")
    order = sorted(by_disp)
    sgd = [d for d in order if "sgd_momentum" in names[d]]
    sgd = [d for k, d in enumerate(sgd) if k + 1 == len(sgd) or sgd[k + 1] - d > 16]  # last of a group
    lo, hi = sgd[-2], sgd[-1]
    return [(names[d], by_disp[d]) for d in order if lo < d <= hi]


def last_step_us(pass_dir):
    """Kernel time per family in the same last step, from the pass's kernel trace (kernels
    serialized under counter collection: isolated durations)."""
    files = glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return {}
    rows = sorted(csv.DictReader(open(files[0])), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("drn::", "") for r in rows]
    sgd = [i for i, n in enumerate(names) if "sgd_momentum" in n]
    sgd = [d for k, d in enumerate(sgd) if k + 1 == len(sgd) or sgd[k + 1] - d > 16]
    if len(sgd) < 2:
        return {}
    us = collections.defaultdict(float)
    for i in range(sgd[-2] + 1, sgd[-1] + 1):
        r = rows[i]
        us[names[i].split("<")[0]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return us


def main():
    out = sys.argv[1]
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for p in sorted(glob.glob(os.path.join(out, "p*"))):
        if not os.path.isdir(p):
            continue
        for name, ctr in last_step(p):
            key = name.split("<")[0]
            if p.endswith("p0"):
                cnt[key] += 1
            for k, v in ctr.items():
                fam[key][k] += v
    # SQ_VALU_MFMA_BUSY_CYCLES sums MFMA-busy cycles over all 1024 SIMDs (16 per 16x16x32 bf16
    # MFMA, checked against SQ_INSTS_MFMA); GRBM_GUI_ACTIVE sums busy cycles over the 8 XCDs
    us = last_step_us(os.path.join(out, "p1"))
    print(f"{'kernel family':28s} {'n':>4s} {'MFMA util%':>10s} {'LDS confl%':>10s} {'VALU/MFMA':>9s} {'HBM MB':>8s}"
          f" {'us':>8s} {'GB/s':>7s}")
    for key, c in sorted(fam.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        cycles = c.get("GRBM_GUI_ACTIVE", 0) / 8
        util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1024 * cycles, 1) * 100
        confl = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 0), 1) * 100
        nm = c.get("SQ_INSTS_MFMA", 0)
        vm = f"{c.get('SQ_INSTS_VALU', 0) / nm:9.1f}" if nm else f"{'-':>9s}"
        mb = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e6
        t = us.get(key, 0.0)
        bw = f"{mb / t * 1e3:7.0f}" if t > 0 else f"{'-':>7s}"
        print(f"{key[:28]:28s} {cnt[key]:4d} {util:10.1f} {confl:10.1f} {vm} {mb:8.0f} {t:8.0f} {bw}")


if __name__ == "__main__":
    main()
