#!/usr/bin/env python3
"""Halo-tiled 3x3 conv (conv_halo.hip) vs the implicit-GEMM family on the ResNet-50 stride-1
3x3 layers at batch 128: forward (BN-statistics epilogue) and data-gradient (fused BN-backward
epilogue) modes. Interleaved timing in one process; prints one JSON line per layer/mode.

usage: halo_bench.py [batch] [iters]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
be = HipBackend("cuda")
L = be.L
h0 = L.drn_conv_halo_cfg0()
LAYERS = [(56, 64), (28, 128), (14, 256), (7, 512)]


def timed(a, n):
    s = be.stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    assert L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), s) == 0
    e0.record()
    for _ in range(n):
        L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), s)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for H, C in LAYERS:
    for mode in ("fwd", "dgrad"):
        torch.manual_seed(0)
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(C, 3, 3, C, device="cuda") * (2.0 / (9 * C)) ** 0.5).bfloat16()
        y = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(8, 2, C, device="cuda")
        g = ConvGeom(1, 1, 1)
        bb = None
        if mode == "dgrad":
            bb = (torch.randn(N, H, H, C, device="cuda").bfloat16(), torch.rand(C, device="cuda") + 0.5,
                  torch.randn(C, device="cuda"), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"))
        a = be.conv_args(x, w, y, g, stats=st, bn_bwd=bb)
        key = be.conv_key(a)
        os.environ["DRN_CONV_CANDS"] = ",".join(str(c) for c in [100] + list(range(L.drn_conv_glds_num_cfgs())))
        old_cfg = be._tune_conv(a, key)
        del os.environ["DRN_CONV_CANDS"]
        a.cfg = old_cfg[0]
        be._set_ksplit(a, old_cfg[1])
        res = {"H": H, "C": C, "N": N, "mode": mode, "old_cfg": list(old_cfg)}
        flops = 2.0 * N * H * H * C * 9 * C
        cands = {"old": old_cfg}
        for i in range(L.drn_conv_halo_num_cfgs()):
            cands[f"halo{i}"] = (h0 + i, 1)
        best = {k: float("inf") for k in cands}
        for _ in range(3):  # interleaved rounds
            for k, (cfg, ks) in cands.items():
                a.cfg = cfg
                be._set_ksplit(a, ks)
                if L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), be.stream()) != 0:
                    best[k] = None
                    continue
                if best[k] is not None:
                    best[k] = min(best[k], timed(a, ITERS))
        for k, us in best.items():
            res[k] = None if us is None else {"us": round(us, 1), "tfs": round(flops / us / 1e6, 0)}
        print(json.dumps(res), flush=True)
