#!/usr/bin/env python3
"""Vendor-library ceiling per ResNet-50 conv shape (measurement only, never a product path).

For every distinct forward conv geometry of ResNet-50 v2 at batch N (bf16, NHWC), times:
  ours  -- the in-tree HIP kernels, autotuned over every configuration (plain conv: no BN
           prologue / residual / statistics, so it is the same op the library runs);
  blas  -- 1x1 stride-1 layers as one GEMM [M, C] x [C, K] via torch.matmul (hipBLASLt);
  miopen-- every layer via F.conv2d on channels_last bf16 tensors (MIOpen's own autotuned find).
Prints one JSON line per geometry and a totals line. Used to tell whether a shape is hard for
any kernel on this chip (small N / K for 256 CUs) or only for ours.

usage: lib_ceiling.py [batch] [iters]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_resnet_tensorflow_amd.models.spec import build_spec  # noqa: E402
from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.backends.cudnn.benchmark = True


def timeit(fn, n=ITERS):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best


sp = build_spec("imagenet", 50)
geoms = {}
for b in sp.blocks:
    h = b.in_hw
    convs = ([b.proj] if b.proj is not None else []) + list(b.convs)
    for i, c in enumerate(convs):
        hin = b.in_hw if (b.proj is not None and i == 0) else h
        key = (c.k, c.cin_store, c.cout, hin, c.stride)
        geoms.setdefault(key, 0)
        geoms[key] += 1
        if not (b.proj is not None and i == 0):
            h = c.out_hw(h)

be = HipBackend("cuda")
tot = {"ours": 0.0, "blas": 0.0, "miopen": 0.0}
for (k, C, K, H, s), count in sorted(geoms.items()):
    pad = k // 2
    P = (H + 2 * pad - k) // s + 1
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, k, k, C, device="cuda") * (2.0 / (k * k * C)) ** 0.5).bfloat16()
    y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
    a = be.conv_args(x, w, y, ConvGeom(s, pad, pad))
    cfg = be._tune_conv(a, be.conv_key(a))
    a.cfg = cfg[0]
    be._set_ksplit(a, cfg[1])
    st = be.stream()
    ours = timeit(lambda: be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), st))
    flops = 2.0 * N * P * P * K * k * k * C
    row = {"k": k, "C": C, "K": K, "H": H, "stride": s, "count": count, "cfg": list(cfg),
           "ours_us": round(ours, 1), "ours_tfs": round(flops / ours / 1e6)}
    tot["ours"] += ours * count
    if k == 1 and s == 1:
        xm, wm = x.view(-1, C), w.view(K, C).t()
        blas = timeit(lambda: torch.matmul(xm, wm))
        row.update(blas_us=round(blas, 1), blas_tfs=round(flops / blas / 1e6))
        tot["blas"] += blas * count
    else:
        tot["blas"] += ours * count  # no plain-GEMM form: counted at our time
    xc = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
    wc = w.permute(0, 3, 1, 2)
    try:
        mi = timeit(lambda: F.conv2d(xc, wc, stride=s, padding=pad))
        row.update(miopen_us=round(mi, 1), miopen_tfs=round(flops / mi / 1e6))
        tot["miopen"] += mi * count
    except RuntimeError as e:  # pragma: no cover - library refusal is a result, not a failure
        row["miopen_err"] = str(e)[:80]
    print(json.dumps(row), flush=True)
print(json.dumps({"total_fwd_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)
