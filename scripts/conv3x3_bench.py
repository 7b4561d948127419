#!/usr/bin/env python3
"""The ResNet-50 bs128 stride-1 3x3 convolutions in isolation: every LDS-DMA configuration (and
the register-staged kernel) timed on each shape, plain (forward) and with the fused BN-backward
epilogue (the data gradient's form); prints the best configuration's time and TF/s per shape.
Run it against two kernel libraries (DRN_KERNEL_LIB) to A/B a main-loop change.

    python scripts/conv3x3_bench.py [--batch 128] [--iters 20]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend


def timeit(fn, iters):
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
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--all", action="store_true", help="print every configuration's time")
    a = ap.parse_args()
    be = HipBackend()
    be.autotune = False
    cfgs = [100] + list(range(be.L.drn_conv_glds_num_cfgs()))
    out = []
    for H, C in ((56, 64), (28, 128), (14, 256), (7, 512)):
        N = a.batch
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        bx = torch.randn(N, H, H, C, device="cuda").bfloat16()
        st = torch.zeros(be.stats_replicas, 2, C, device="cuda")
        v = [torch.rand(C, device="cuda") + 0.5 for _ in range(4)]
        g = ConvGeom(1, 1, 1)
        flop = 2.0 * N * H * H * C * C * 9
        for name, kw in (("fwd", {}), ("bnbwd", dict(stats=st, bn_bwd=(bx, v[0], v[1], v[2], v[3])))):
            best = (float("inf"), None)
            for cfg in cfgs:
                args = be.conv_args(x, w, y, g, **kw)
                args.cfg = cfg
                if be.L.drn_conv_fwd2(ctypes.byref(args), be.zero_page.data_ptr(), be.stream()) != 0:
                    continue
                t = timeit(lambda: be.launch_conv(args), a.iters)
                if a.all:
                    print(f"   {H:2d}x{H:<2d} {name:5s} cfg {cfg:3d} {t:7.1f} us", flush=True)
                best = min(best, (t, cfg))
            t, cfg = best
            print(f"{H:2d}x{H:<2d} {C:3d}->{C:3d} {name:5s} best cfg {cfg:3d} {t:7.1f} us {flop / t / 1e6:6.0f} TF/s",
                  flush=True)
            out.append({"H": H, "C": C, "mode": name, "cfg": cfg, "us": round(t, 2), "tflops": round(flop / t / 1e6)})
    if a.json:
        json.dump(out, open(a.json, "w"))


if __name__ == "__main__":
    main()
