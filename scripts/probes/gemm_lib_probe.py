#!/usr/bin/env python3
"""Library-GEMM probe: torch.matmul (hipBLASLt) bf16 time for every ResNet-50 (bs 128) 1x1
convolution viewed as a plain GEMM [M pixels x Cin] @ [Cin x Cout], next to the achieved
HBM bandwidth / MFMA rate -- the yardstick for the in-tree fused 1x1 conv kernels (whose
per-layer times are in profiles/r2_rn50_bs128_op_breakdown_final.txt)."""
import json
import sys

import torch

SHAPES = [  # (label, M, Cin, Cout)
    ("s1 64->256 @56", 128 * 56 * 56, 64, 256),
    ("s1 256->64 @56", 128 * 56 * 56, 256, 64),
    ("s1 64->64 @56", 128 * 56 * 56, 64, 64),
    ("s2 256->128 @56", 128 * 56 * 56, 256, 128),
    ("s2 128->512 @28", 128 * 28 * 28, 128, 512),
    ("s2 512->128 @28", 128 * 28 * 28, 512, 128),
    ("s3 512->256 @28", 128 * 28 * 28, 512, 256),
    ("s3 256->1024 @14", 128 * 14 * 14, 256, 1024),
    ("s3 1024->256 @14", 128 * 14 * 14, 1024, 256),
    ("s4 1024->512 @14", 128 * 14 * 14, 1024, 512),
    ("s4 512->2048 @7", 128 * 7 * 7, 512, 2048),
    ("s4 2048->512 @7", 128 * 7 * 7, 2048, 512),
]


def main():
    dev = "cuda"
    out = []
    for label, M, K, N in SHAPES:
        a = torch.randn(M, K, device=dev).bfloat16()
        b = torch.randn(K, N, device=dev).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        r = torch.randn(M, N, device=dev).bfloat16()
        for _ in range(5):
            torch.matmul(a, b, out=c)
        torch.cuda.synchronize()
        res = {}
        for name, fn in (("mm", lambda: torch.matmul(a, b, out=c)),
                         ("addmm_res", lambda: torch.addmm(r, a, b, out=c))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            byts = 2 * (M * K + K * N + M * N * (2 if name == "addmm_res" else 1))
            res[name] = dict(us=round(us, 1), tbs=round(byts / us / 1e6, 2), tfs=round(2 * M * K * N / us / 1e6, 1))
        out.append(dict(label=label, M=M, K=K, N=N, **res))
        print(json.dumps(out[-1]), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
