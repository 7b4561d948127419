#!/usr/bin/env python3
"""Per-launch roofline of the convolution kernels in one profiled training step.

Replays the executor's launch sequence on a recording backend (CPU, no kernels run) to get
each conv launch's geometry, zips it with the conv kernels of the last step in a rocprofv3
kernel trace, and prints time, TFLOP/s and minimal-traffic TB/s per launch class.
usage: scripts/conv_roofline.py <kernel_trace.csv> [--dataset imagenet --batch 128]"""
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

    def conv_fwd(self, x, w, y, g, in_bn=None, relu_in=True, residual=None, stats=None, out_map=None, bn_bwd=None,
                 **kw):
        K, R, S, C = w.shape
        P, Q = (out_map.P, out_map.Q) if out_map is not None else (y.shape[1], y.shape[2])
        M = x.shape[0] * P * Q
        self.log.append(("conv", M, K, R * S * C, x.numel() * 2 + y.numel() * 2 * (1 + (residual is not None))))

    def conv_wgrad(self, x, dy, out, g, in_bn=None, relu_in=True, ws=None, **kw):
        K, R, S, C = out.shape
        M = dy.shape[0] * dy.shape[1] * dy.shape[2]
        self.log.append(("wgrad", M, K, R * S * C, x.numel() * 2 + dy.numel() * 2))


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
    kconv = [r for r in step if "conv_fwd" in r["Kernel_Name"]]
    kwg = [r for r in step if "conv_wgrad" in r["Kernel_Name"]]
    be = Rec()
    spec = build_spec(a.dataset, 50)
    with torch.no_grad():
        ex = Executor(spec, 2, be, "cpu", seed=0)  # geometry scales with N: record at N=2, rescale
        be.log.clear()
        ex.forward(True)
        ex.backward()
    scale = a.batch / 2
    convs = [l for l in be.log if l[0] == "conv"]
    wgs = [l for l in be.log if l[0] == "wgrad"]
    assert len(convs) == len(kconv), (len(convs), len(kconv))
    assert len(wgs) == len(kwg), (len(wgs), len(kwg))
    cls = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    tot = 0.0
    for (kind, M, K, Kt, by), r in list(zip(convs, kconv)) + list(zip(wgs, kwg)):
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        M = int(M * scale)
        fl = 2.0 * M * K * Kt
        key = (kind, "1x1" if Kt == K and False else "", f"M{M}", f"K{K}", f"Kt{Kt}")
        c = cls[(kind, M, K, Kt)]
        c[0] += t
        c[1] += fl
        c[2] += by * scale
        c[3] += 1
        tot += t
    print(f"{'kind':6s} {'M':>8s} {'K':>5s} {'Ktot':>5s} {'n':>3s} {'us':>8s} {'TF/s':>6s} {'TB/s':>6s}")
    for (kind, M, K, Kt), (t, fl, by, n) in sorted(cls.items(), key=lambda kv: -kv[1][0]):
        print(f"{kind:6s} {M:8d} {K:5d} {Kt:5d} {n:3d} {t:8.1f} {fl / t / 1e6:6.0f} {by / t / 1e6:6.2f}")
    print(f"total conv+wgrad us/step: {tot:.0f}")


if __name__ == "__main__":
    main()
