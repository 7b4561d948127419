#!/usr/bin/env python3
"""Epilogue-cost microbenchmark: one conv geometry timed with/without BN statistics, residual
and the fused BN-backward reduction (event timing over back-to-back launches)."""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="128,56,64,256,1;128,56,256,64,1;128,14,256,1024,1;128,14,256,256,3")
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--cfgs", default="", help="comma list: sweep configurations, print TB/s per variant")
    a = ap.parse_args()
    be = HipBackend()
    be.autotune = False
    for sh in a.shapes.split(";"):
        N, H, C, K, R = map(int, sh.split(","))
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, H, H, K, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(N, H, H, K, device="cuda").bfloat16()
        bx = torch.randn(N, H, H, K, device="cuda").bfloat16()
        st = torch.zeros(be.stats_replicas, 2, K, device="cuda")
        v = [torch.rand(K, device="cuda") for _ in range(4)]
        g = ConvGeom(1, (R - 1) // 2, (R - 1) // 2)
        xb, yb = x.numel() * 2, y.numel() * 2
        nbytes = {"plain": xb + yb, "stats": xb + yb, "res": xb + 2 * yb, "res+stats": xb + 2 * yb, "bnbwd": xb + 2 * yb}
        if a.cfgs:
            for cfg in [int(c) for c in a.cfgs.split(",")]:
                line = []
                for name, kw in (("plain", {}), ("res+stats", dict(residual=r, stats=st))):
                    args = be.conv_args(x, w, y, g, **kw)
                    args.cfg = cfg
                    if be.L.drn_conv_fwd2(__import__("ctypes").byref(args), be.zero_page.data_ptr(), be.stream()) != 0:
                        line = None
                        break
                    t = timeit(lambda: be.launch_conv(args))
                    line.append(f"{name} {t:7.1f}us {nbytes[name] / t / 1e6:5.2f}TB/s")
                if line:
                    print(f"N{N} {H}x{H} {C}->{K} k{R} cfg{cfg:3d}: " + "  ".join(line), flush=True)
            continue
        res = {}
        for name, kw in (("plain", {}), ("stats", dict(stats=st)), ("res", dict(residual=r)),
                         ("res+stats", dict(residual=r, stats=st)),
                         ("bnbwd", dict(stats=st, bn_bwd=(bx, v[0], v[1], v[2], v[3])))):
            args = be.conv_args(x, w, y, g, **kw)
            if a.cfg >= 0:
                args.cfg = a.cfg
            res[name] = timeit(lambda: be.launch_conv(args))
        fl = 2.0 * N * H * H * K * R * R * C
        print(f"N{N} {H}x{H} {C}->{K} k{R}: " + "  ".join(f"{k} {t:.1f}us" for k, t in res.items()) +
              f"  (plain {fl / res['plain'] / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
