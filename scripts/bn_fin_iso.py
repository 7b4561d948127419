#!/usr/bin/env python3
"""Isolated time of the finalizing BatchNorm backward apply (bn.hip bn_bwd_apply_fin_kernel) and
forward apply (bn_apply_fin_kernel) on the ResNet-50 bs128 shapes, best of 3 x 50 launches.
Compare two kernel libraries by running it twice (DRN_KERNEL_LIB=<variant .so> for the other).

    python scripts/bn_fin_iso.py [--tag NAME]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ops.backend import BnCfin, HipBackend  # noqa: E402

SHAPES = [(128 * 56 * 56, 64), (128 * 56 * 56, 256), (128 * 28 * 28, 128), (128 * 28 * 28, 512),
          (128 * 14 * 14, 256), (128 * 7 * 7, 512)]


def best_us(fn, n=50, rounds=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.environ.get("DRN_KERNEL_LIB", "tree"))
    a = ap.parse_args()
    be = HipBackend("cuda")
    torch.manual_seed(0)
    for M, C in SHAPES:
        x = torch.randn(M, C, device="cuda").bfloat16()
        dy = torch.randn(M, C, device="cuda").bfloat16()
        add = torch.randn(M, C, device="cuda").bfloat16()
        dx = torch.empty_like(x)
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
        mu, isd = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
        bst = torch.randn(1, 2, C, device="cuda")
        gamma = torch.rand(C, device="cuda") + 0.5
        dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        fin = BnCfin(bst, float(M), gamma, mean=mu, invstd=isd, dgamma=dg, dbeta=db, publish=True)
        t0 = best_us(lambda: be.bn_bwd_apply_fin(dy, None, 0, x, sc, sh, fin, None, dx, relu=True))
        t1 = best_us(lambda: be.bn_bwd_apply_fin(dy, None, 0, x, sc, sh, fin, add, dx, relu=True))
        gb = M * C * 2 * 3 / 1e6  # bytes / us -> TB/s
        print(f"{a.tag:>12} bwd_apply_fin M={M:>7} C={C:>4}: {t0:7.2f} us ({gb / t0:5.2f} TB/s)  "
              f"+add {t1:7.2f} us ({gb * 4 / 3 / t1:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
