#!/usr/bin/env python3
"""Per-layer roofline of the forward convs of one profiled ResNet-50 step.

usage: fwd_roofline.py <kernel_trace.csv> [batch]
Matches the step's conv_fwd launches (in issue order) to the executor's forward conv order
(stem, then per block: projection, conv1, conv2, conv3) and prints, per layer, FLOPs, the
minimum HBM bytes (input once, output once, residual once; bf16), the measured time and
the roofline time max(bytes / 5.5 TB/s, FLOPs / 1.3 PF/s).
"""
import csv
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributed_resnet_tensorflow_amd.models.spec import build_spec  # noqa: E402

BW, PF = 5.5e12, 1.3e15
rows = list(csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 128
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 16]
step = rows[idx[-2] + 1:idx[-1] + 1]
convs = []
for r in step:
    if "softmax" in r["Kernel_Name"]:
        break
    if "conv_fwd" in r["Kernel_Name"] or "conv_nk" in r["Kernel_Name"]:
        convs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
sp = build_spec("imagenet", 50)
layers = [("stem", sp.stem, sp.image_size, False)]
for b in sp.blocks:
    if b.proj is not None:
        layers.append((f"s{b.stage}b{b.index} proj", b.proj, b.in_hw, False))
    h = b.in_hw
    for i, c in enumerate(b.convs):
        layers.append((f"s{b.stage}b{b.index} conv{i + 1}", c, h, i == len(b.convs) - 1))
        h = c.out_hw(h)
tot_m = tot_r = 0.0
print(f"{'layer':16s} {'k':>2s} {'cin':>5s} {'cout':>5s} {'hw':>4s} {'GFLOP':>7s} {'MB':>7s} {'us':>7s} {'roof':>7s} {'TF/s':>6s} {'TB/s':>6s}")
for (name, c, h, res), us in zip(layers, convs):
    oh = c.out_hw(h)
    M = N * oh * oh
    fl = 2.0 * M * c.cout * c.k * c.k * c.cin_store
    by = 2.0 * (N * h * h * c.cin_store + M * c.cout * (2 if res else 1))
    roof = max(by / BW, fl / PF) * 1e6
    tot_m += us
    tot_r += roof
    print(f"{name:16s} {c.k:2d} {c.cin:5d} {c.cout:5d} {oh:4d} {fl / 1e9:7.1f} {by / 1e6:7.1f} {us:7.1f} {roof:7.1f} "
          f"{fl / us / 1e6:6.0f} {by / us / 1e6:6.2f}")
print(f"total conv forward {tot_m:.0f} us, roofline {tot_r:.0f} us ({len(convs)} launches, {len(layers)} layers)")
