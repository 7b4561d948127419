#!/usr/bin/env python3
"""Launch one ResNet-50 3x3 layer (batch 128) with a fixed kernel configuration a few times, for
rocprofv3 --pmc passes. usage: halo_pmc_run.py <H> <C> <cfg> [mode fwd|dgrad] [reps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend  # noqa: E402

H, C, cfg = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mode = sys.argv[4] if len(sys.argv) > 4 else "fwd"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
N = 128
be = HipBackend("cuda")
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
w = (torch.randn(C, 3, 3, C, device="cuda") * (2.0 / (9 * C)) ** 0.5).bfloat16()
y = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
st = torch.zeros(8, 2, C, device="cuda")
bb = None
if mode == "dgrad":
    bb = (torch.randn(N, H, H, C, device="cuda").bfloat16(), torch.rand(C, device="cuda") + 0.5,
          torch.randn(C, device="cuda"), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"))
a = be.conv_args(x, w, y, ConvGeom(1, 1, 1), stats=st, bn_bwd=bb)
a.cfg = cfg
for _ in range(reps):
    assert be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), be.stream()) == 0
torch.cuda.synchronize()
print("ok", H, C, cfg, mode)
