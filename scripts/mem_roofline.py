#!/usr/bin/env python3
"""Per-launch bandwidth of the memory-bound kernels (BN apply / BN backward apply / max-pool
backward) in one profiled training step: replays the executor on a recording backend (CPU, no
kernels run) for each launch's byte count, zips it with the kernel trace of the last step.
usage: scripts/mem_roofline.py <kernel_trace.csv> [--dataset imagenet --batch 128]"""
import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor


class Rec(RefBackend):
    def __init__(self):
        super().__init__()
        self.log = []

    def bn_apply(self, x, y, scale, shift, relu=True):
        self.log.append(("bn_apply_kernel", x.numel(), x.numel() * 2 * 2, tuple(x.shape)))

    def bn_bwd_apply(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, coef, add, dx, relu=True):
        n = x.numel()
        b = n * 2 * 3 + (n * 2 if add is not None else 0)
        self.log.append(("bn_bwd_apply_kernel", n, b, tuple(x.shape)))

    def maxpool_bwd(self, dy, arg, dx, k, stride, pad_h, pad_w):
        self.log.append(("maxpool_bwd_kernel", dx.numel(), dy.numel() * 3 + dx.numel() * 2, tuple(dx.shape)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--dataset", default="imagenet")
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
    # a step may update in two launches (backward(defer_tail)): the step ends at the LAST of
    # a group of optimizer launches a few kernels apart
    idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
    step = rows[idx[-2] + 1:idx[-1] + 1]
    be = Rec()
    spec = build_spec(a.dataset, 50)
    with torch.no_grad():
        ex = Executor(spec, 2, be, "cpu", seed=0)
        be.log.clear()
        ex.forward(True)
        ex.backward()
    scale = a.batch / 2
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for name in ("bn_apply_kernel", "bn_bwd_apply_kernel", "maxpool_bwd_kernel"):
        ks = [r for r in step if f"::{name}(" in r["Kernel_Name"] or f"::{name}<" in r["Kernel_Name"]]
        ls = [l for l in be.log if l[0] == name]
        if len(ks) != len(ls):
            print(f"{name}: {len(ks)} kernels vs {len(ls)} launches recorded; skipping")
            continue
        for k, l in zip(ks, ls):
            us = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
            key = (name, l[3][1:])
            agg[key][0] += 1
            agg[key][1] += us
            agg[key][2] += l[2] * scale
    print(f"{'kernel':22s} {'shape(HWC)':>18s} {'n':>3s} {'us':>8s} {'TB/s':>6s}")
    tot = 0.0
    for (name, shp), (n, us, b) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tot += us
        print(f"{name:22s} {str(shp):>18s} {n:3d} {us:8.1f} {b / us / 1e6:6.2f}")
    print(f"total us/step: {tot:.0f}")


if __name__ == "__main__":
    main()
