#!/usr/bin/env python3
"""A/B of the conv epilogue variants on one geometry: no stats / stats with R replicas /
residual, per kernel config. usage: stats_ab.py H C K R stride [cfg...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


H, C, K, R, st = (int(v) for v in sys.argv[1:6])
cfgs = [int(v) for v in sys.argv[6:]] or [0, 3, 20]
N = 128
be = HipBackend()
be.autotune = False
P = H // st
g = ConvGeom(st, (R - 1) // 2, (R - 1) // 2)
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
res = torch.randn_like(y)
sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
for cfg in cfgs:
    be.forced_cfg = cfg
    out = []
    for name, kw in [("plain", {}), ("pro", dict(in_bn=(sc, sh))),
                     ("stats1", dict(stats=torch.zeros(1, 2, K, device="cuda"))),
                     ("stats8", dict(stats=torch.zeros(8, 2, K, device="cuda"))),
                     ("stats64", dict(stats=torch.zeros(64, 2, K, device="cuda"))),
                     ("res", dict(residual=res)),
                     ("pro+res+stats8", dict(in_bn=(sc, sh), residual=res, stats=torch.zeros(8, 2, K, device="cuda")))]:
        try:
            t = timeit(lambda: be.conv_fwd(x, w, y, g, **kw))
        except Exception as ex:  # config not applicable
            t = float("nan")
        out.append(f"{name}:{t:.1f}")
    print(f"H{H} C{C} K{K} R{R} s{st} cfg{cfg}: " + " ".join(out), flush=True)
