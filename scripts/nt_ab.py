#!/usr/bin/env python3
"""A/B of the conv kernel cache-policy switches (drn_conv_set_flags) on training-like layers:
bit0 nt output stores, bit1 nt epilogue loads, bit2 nt activation DMA, bit3 nt weight DMA."""
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


N = 128
be = HipBackend()
LAYERS = [  # H, C, K, R, stride, pro, res, stats
    (56, 64, 256, 1, 1, True, True, True),
    (56, 256, 64, 1, 1, True, False, True),
    (14, 256, 1024, 1, 1, True, True, True),
    (14, 256, 256, 3, 1, False, False, True),
    (28, 128, 128, 3, 1, False, False, True),
    (56, 64, 64, 3, 1, False, False, True),
    (7, 512, 512, 3, 1, True, False, True),
]
FLAGS = [0, 1, 2, 3, 4, 8, 12, 15]
for (H, C, K, R, st, pro, res, stats) in LAYERS:
    P = H // st
    g = ConvGeom(st, (R - 1) // 2, (R - 1) // 2)
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
    y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
    kw = {}
    if pro:
        kw["in_bn"] = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
    if res:
        kw["residual"] = torch.randn_like(y)
    if stats:
        kw["stats"] = torch.zeros(8, 2, K, device="cuda")
    be.L.drn_conv_set_flags(0)
    be.conv_fwd(x, w, y, g, **kw)  # autotune once with default policy
    out = []
    for f in FLAGS:
        be.L.drn_conv_set_flags(f)
        out.append(f"{f}:{timeit(lambda: be.conv_fwd(x, w, y, g, **kw)):.1f}")
    be.L.drn_conv_set_flags(0)
    print(f"H{H} C{C} K{K} R{R} pro{int(pro)} res{int(res)} cfg{be.tune_log[-1][1]}: " + " ".join(out), flush=True)
