#!/usr/bin/env python3
"""Per-layer microbenchmark of the gfx950 kernels on the real network shapes.

For every distinct conv of the chosen network (bs 128 by default) times forward (with the
fused BN prologue + stats epilogue as used in training), data-gradient and weight-gradient
(incl. split-K reduce), plus the BN backward kernels, and prints achieved TFLOP/s and the
effective HBM bandwidth of the minimal tensor traffic. usage:
  python scripts/kernel_bench.py [--dataset imagenet] [--batch 128] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend, dgrad_geom


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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="imagenet")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--only", default="", help="substring filter on the layer name (e.g. 'conv 256->256 k3s1')")
    ap.add_argument("--pro", action="store_true", help="fused BN prologue in fwd/wgrad (default: materialized)")
    ap.add_argument("--sweep", action="store_true", help="time every conv kernel config for fwd and dgrad")
    ap.add_argument("--no_bn", action="store_true")
    a = ap.parse_args()
    spec = build_spec(a.dataset, a.resnet_size)
    be = HipBackend()
    N = a.batch
    shapes = {}
    hw = spec.stem_hw
    h_in = spec.image_size
    shapes[("stem", spec.stem.cin_store, spec.stem.cout, spec.stem.k, spec.stem.stride, h_in)] = 1
    for blk in spec.blocks:
        h = blk.in_hw
        if blk.proj is not None:
            c = blk.proj
            shapes[("proj", c.cin, c.cout, 1, c.stride, h)] = shapes.get(("proj", c.cin, c.cout, 1, c.stride, h), 0) + 1
        for c in blk.convs:
            k = ("conv", c.cin, c.cout, c.k, c.stride, h)
            shapes[k] = shapes.get(k, 0) + 1
            h = c.out_hw(h)
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "bn_bwd": 0.0}
    for (kind, cin, cout, k, s, H), cnt in shapes.items():
        if a.only and a.only not in f"{kind} {cin}->{cout} k{k}s{s} @{H}":
            continue
        P = H if s == 1 else (H - 1) // s + 1
        g = ConvGeom(s, (k - 1) // 2, (k - 1) // 2)
        x = torch.randn(N, H, H, cin, device="cuda").bfloat16()
        w = (torch.randn(cout, k, k, cin, device="cuda") * 0.05).bfloat16()
        wt = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        y = torch.empty(N, P, P, cout, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(N, P, P, cout, device="cuda").bfloat16()
        dx = torch.empty_like(x)
        sc, sh = torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.1
        st = torch.zeros(2, cout, device="cuda")
        dw = torch.empty(cout, k, k, cin, device="cuda")
        ws = torch.empty(max(16, be.wgrad_ws_elems(N * P * P, cout, k, k, cin)), device="cuda")
        pro = (sc, sh) if (a.pro and kind != "stem") else None
        flops = 2.0 * N * P * P * cout * k * k * cin
        t_f = timeit(lambda: be.conv_fwd(x, w, y, g, in_bn=pro, stats=st), a.iters)
        t_w = timeit(lambda: be.conv_wgrad(x, dy, dw, g, in_bn=pro, ws=ws), a.iters)
        t_d = timeit(lambda: be.conv_fwd(dy, wt, dx, dgrad_geom(g, k, k)), a.iters) if kind != "stem" else 0.0
        if a.sweep:
            from distributed_resnet_tensorflow_amd.ops.backend import dgrad_geom as _dg
            res_f, res_d = [], []
            for cfg in [100] + list(range(be.L.drn_conv_glds_num_cfgs())):
                af = be.conv_args(x, w, y, g, in_bn=pro, stats=st)
                af.cfg = cfg
                res_f.append((timeit(lambda: be.launch_conv(af), a.iters), cfg))
                if kind != "stem" and s == 1:
                    ad = be.conv_args(dy, wt, dx, _dg(g, k, k))
                    ad.cfg = cfg
                    res_d.append((timeit(lambda: be.launch_conv(ad), a.iters), cfg))
            res_w = []
            for ns in (0, 2, 3):
                be.forced_wgrad_ns = ns
                res_w.append((timeit(lambda: be.conv_wgrad(x, dy, dw, g, in_bn=pro, ws=ws), a.iters), ns))
            be.forced_wgrad_ns = None
            fmt = lambda r: " ".join(f"{c}:{t:.0f}" for t, c in r)
            print(f"      wgrad best {min(res_w)} | {fmt(res_w)}", flush=True)
            print(f"sweep {kind} {cin}->{cout} k{k}s{s} @{H} x{cnt}: fwd best {min(res_f)} | {fmt(res_f)}", flush=True)
            if res_d:
                print(f"      dgrad best {min(res_d)} | {fmt(res_d)}", flush=True)
        bx, by = x.numel() * 2, y.numel() * 2
        r = dict(kind=kind, cin=cin, cout=cout, k=k, s=s, H=H, count=cnt,
                 fwd_us=t_f, fwd_tf=flops / t_f / 1e6, fwd_gbs=(bx + by) / t_f / 1e3,
                 wgrad_us=t_w, wgrad_tf=flops / t_w / 1e6, wgrad_gbs=(bx + by) / t_w / 1e3,
                 dgrad_us=t_d, dgrad_tf=(flops / t_d / 1e6) if t_d else 0, dgrad_gbs=((bx + by) / t_d / 1e3) if t_d else 0)
        rows.append(r)
        tot["fwd"] += t_f * cnt
        tot["wgrad"] += t_w * cnt
        tot["dgrad"] += t_d * cnt
        del x, w, wt, y, dy, dx, dw, ws
    print(f"{'layer':34s} {'cnt':>3} | {'fwd us':>8} {'TF/s':>6} {'GB/s':>6} | {'dgrad us':>8} {'TF/s':>6} {'GB/s':>6} | "
          f"{'wgrad us':>8} {'TF/s':>6} {'GB/s':>6}")
    for r in rows:
        name = f"{r['kind']} {r['cin']}->{r['cout']} k{r['k']}s{r['s']} @{r['H']}"
        print(f"{name:34s} {r['count']:>3} | {r['fwd_us']:8.1f} {r['fwd_tf']:6.0f} {r['fwd_gbs']:6.0f} | "
              f"{r['dgrad_us']:8.1f} {r['dgrad_tf']:6.0f} {r['dgrad_gbs']:6.0f} | {r['wgrad_us']:8.1f} {r['wgrad_tf']:6.0f} "
              f"{r['wgrad_gbs']:6.0f}")
    print("totals per step (us):", {k: round(v, 1) for k, v in tot.items()})
    # BN backward kernels on the largest activation shapes
    for (C, H) in (() if a.no_bn else ((64, 56), (256, 56), (128, 28), (512, 28), (1024, 14), (2048, 7))):
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        da = torch.randn_like(x)
        out = torch.empty_like(x)
        v = [torch.rand(C, device="cuda") for _ in range(4)]
        part = torch.zeros(2, C, device="cuda")
        coef = torch.rand(3 * C, device="cuda")
        t_r = timeit(lambda: be.bn_bwd_reduce(da, None, 0, x, v[0], v[1], v[2], v[3], part), a.iters)
        t_a = timeit(lambda: be.bn_bwd_apply(da, None, 0, x, v[0], v[1], v[2], v[3], coef, da, out), a.iters)
        nb = x.numel() * 2
        print(f"bn C={C} @{H}: reduce {t_r:7.1f} us ({2 * nb / t_r / 1e3:5.0f} GB/s)  apply+add {t_a:7.1f} us "
              f"({4 * nb / t_a / 1e3:5.0f} GB/s)")
    if a.json:
        json.dump({"rows": rows, "totals_us": tot}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
