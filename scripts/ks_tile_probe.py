#!/usr/bin/env python3
"""Do split-K / stream-K versions of the 8-wave big tiles (256x128, 128x256, 256x256) win on the
under-filled ResNet-50 grids? Runs the backend's full conv tuner (every configuration, split-K
factors, stream-K grids; DRN_TUNE_DB=off) on the stage-3/4 forward and data-gradient shapes of the
bs128 step and prints the winner and its time per geometry. Run it once per kernel library
(DRN_KERNEL_LIB) to compare.

    DRN_KERNEL_LIB=<lib> python scripts/ks_tile_probe.py [--json out]
"""
import argparse
import json
import os
import sys

os.environ["DRN_TUNE_DB"] = "off"
os.environ.setdefault("DRN_TUNE_ITERS", "10")
os.environ.setdefault("DRN_TUNE_ROUNDS", "3")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend  # noqa: E402

# (N, H, C, K, R, stride): forward and data-gradient (C/K swapped) shapes of stages 3 and 4
SHAPES = [(128, 14, 256, 256, 3, 1), (128, 7, 512, 512, 3, 1), (128, 14, 1024, 256, 1, 1),
          (128, 14, 256, 1024, 1, 1), (128, 7, 2048, 512, 1, 1), (128, 7, 512, 2048, 1, 1),
          (128, 28, 128, 128, 3, 1), (128, 28, 512, 128, 1, 1), (128, 28, 128, 512, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    be = HipBackend()
    out = []
    for N, H, C, K, R, st in SHAPES:
        p = (R - 1) // 2
        P = (H + 2 * p - R) // st + 1
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        args = be.conv_args(x, w, y, ConvGeom(st, p, p))
        key = be.conv_key(args)
        best = be._tune_conv(args, key)
        us = be.tune_log[-1][2]
        flop = 2.0 * N * P * P * K * R * R * C
        out.append({"shape": [N, H, C, K, R, st], "cfg": list(best), "us": us, "tflops": round(flop / us / 1e6)})
        print(f"N{N} {H}x{H} {C:5d}->{K:5d} {R}x{R}: best {best} {us:7.1f} us {flop / us / 1e6:6.0f} TF/s", flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"))


if __name__ == "__main__":
    main()
