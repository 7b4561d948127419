#!/usr/bin/env python3
"""What the fused prologues / epilogues cost: every distinct ResNet-50 bs128 convolution timed in
isolation, best configuration per variant, as a plain conv and in the fused forms the training
step launches (statistics epilogue, BN-apply prologue, residual add, BN-backward epilogue).
Prints per layer the time, the compulsory bytes and the achieved streaming rate.

    python scripts/conv_fusion_cost.py [--batch 128] [--iters 20] [--only 1x1|3x3]
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


# (H_in, C, K, kernel, stride): every distinct forward convolution of ResNet-v2-50 (stem excluded)
LAYERS = [
    (56, 64, 64, 1, 1), (56, 64, 256, 1, 1), (56, 256, 64, 1, 1), (56, 256, 128, 1, 1),
    (28, 128, 512, 1, 1), (28, 512, 128, 1, 1), (28, 512, 256, 1, 1),
    (14, 256, 1024, 1, 1), (14, 1024, 256, 1, 1), (14, 1024, 512, 1, 1),
    (7, 512, 2048, 1, 1), (7, 2048, 512, 1, 1),
    (56, 256, 512, 1, 2), (28, 512, 1024, 1, 2), (14, 1024, 2048, 1, 2),
    (56, 64, 64, 3, 1), (28, 128, 128, 3, 1), (14, 256, 256, 3, 1), (7, 512, 512, 3, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--variants", default="", help="comma-separated subset of the variant names")
    ap.add_argument("--layers", default="", help="comma-separated layer indices of LAYERS")
    a = ap.parse_args()
    be = HipBackend()
    be.autotune = False
    cfgs = [100] + list(range(be.L.drn_conv_glds_num_cfgs()))
    out = []
    N = a.batch
    for li, (H, C, K, k, s) in enumerate(LAYERS):
        if a.only and a.only != f"{k}x{k}":
            continue
        if a.layers and str(li) not in a.layers.split(","):
            continue
        P = (H + 2 * (k // 2) - k) // s + 1
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, k, k, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        res = torch.randn(N, P, P, K, device="cuda").bfloat16()
        bx = torch.randn(N, P, P, K, device="cuda").bfloat16()
        st = torch.zeros(be.stats_replicas, 2, K, device="cuda")
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.rand(C, device="cuda") - 0.5
        v = [torch.rand(K, device="cuda") + 0.5 for _ in range(4)]
        g = ConvGeom(s, k // 2, k // 2)
        xb, yb = x.numel() * 2, y.numel() * 2
        variants = (
            ("plain", {}, xb + yb),
            ("stats", dict(stats=st), xb + yb),
            ("pro", dict(in_bn=(sc, sh)), xb + yb),
            ("pro+stats", dict(in_bn=(sc, sh), stats=st), xb + yb),
            ("pro+res+stats", dict(in_bn=(sc, sh), residual=res, stats=st), xb + 2 * yb),
            ("bnbwd", dict(stats=st, bn_bwd=(bx, v[0], v[1], v[2], v[3])), xb + 2 * yb),
            ("stats_rep1", dict(stats=torch.zeros(1, 2, K, device="cuda")), xb + yb),
            ("stats_rep64", dict(stats=torch.zeros(64, 2, K, device="cuda")), xb + yb),
        )
        for name, kw, nbytes in variants:
            if a.variants and name not in a.variants.split(","):
                continue
            best = (float("inf"), None)
            for cfg in cfgs:
                args = be.conv_args(x, w, y, g, **kw)
                args.cfg = cfg
                if be.L.drn_conv_fwd2(ctypes.byref(args), be.zero_page.data_ptr(), be.stream()) != 0:
                    continue
                t = timeit(lambda: be.launch_conv(args), a.iters)
                best = min(best, (t, cfg))
            t, cfg = best
            flop = 2.0 * N * P * P * K * C * k * k
            print(f"{H:3d}^2 {C:4d}->{K:4d} {k}x{k}/{s} {name:14s} cfg {cfg:3d} {t:7.1f} us "
                  f"{nbytes / t / 1e6:5.2f} TB/s {flop / t / 1e6:5.0f} TF/s", flush=True)
            out.append({"H": H, "C": C, "K": K, "k": k, "s": s, "variant": name, "cfg": cfg, "us": round(t, 2),
                        "tbs": round(nbytes / t / 1e6, 3)})
    if a.json:
        json.dump(out, open(a.json, "w"))


if __name__ == "__main__":
    main()
