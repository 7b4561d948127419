#!/usr/bin/env python3
"""Time every conv kernel configuration on one geometry with the training epilogue flags.
usage: cfg_sweep.py N H C K R stride [pro] [res] [stats]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend


def timeit(fn, iters=30):
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


N, H, C, K, R, st = (int(v) for v in sys.argv[1:7])
flags = set(sys.argv[7:])
be = HipBackend()
P = (H + 2 * ((R - 1) // 2) - R) // st + 1
g = ConvGeom(st, (R - 1) // 2, (R - 1) // 2)
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
kw = {}
if "pro" in flags:
    kw["in_bn"] = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
if "res" in flags:
    kw["residual"] = torch.randn_like(y)
if "stats" in flags:
    kw["stats"] = torch.zeros(8, 2, K, device="cuda")
out = []
nk = [be.L.drn_conv_nk_cfg0() + i for i in range(be.L.drn_conv_nk_num_cfgs())] if K in (16, 32) else []
for cfg in [100] + list(range(be.L.drn_conv_glds_num_cfgs())) + nk:
    # split-K factors / stream-K grids (< 0; only the split-capable configurations accept them)
    for ks in (1, 2, 3, 4, -256, -512):
        a = be.conv_args(x, w, y, g, **kw)
        a.cfg = cfg
        be._set_ksplit(a, ks)
        if be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), be.stream()) != 0:
            continue
        t = timeit(lambda: be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), be.stream()))
        out.append((t, f"{cfg}" if ks == 1 else f"{cfg}/k{ks}" if ks > 1 else f"{cfg}/sk{-ks}"))
out.sort()
print(f"N{N} H{H} C{C} K{K} R{R} s{st} {sorted(flags)}: " + " ".join(f"{c}:{t:.1f}" for t, c in out[:14]), flush=True)
