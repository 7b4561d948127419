"""Debug probe: repeated launches of the weight gradient with the in-kernel split-K reduction."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend, RefBackend

hip, ref = HipBackend(), RefBackend("cpu")
for case in [(4, 16, 16, 16, 3, 1, 1), (8, 14, 256, 256, 3, 1, 1)]:
    N, H, C, K, R, s, p = case
    torch.manual_seed(1)
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, H, H, C).bfloat16()
    dy = torch.randn(N, P, P, K).bfloat16()
    g = ConvGeom(s, p, p)
    dw_ref = torch.zeros(K, R, R, C)
    ref.conv_wgrad(x.float(), dy.float(), dw_ref, g)
    ws = torch.zeros(max(1, hip.wgrad_ws_elems(N * P * P, K, R, R, C)), device="cuda")
    for ns in (2, 3):
        dw = torch.full((K, R, R, C), float("nan"), device="cuda")
        xd, dyd = x.cuda(), dy.cuda()   # (raw pointers in the launch arguments: keep them alive)
        a = hip.wgrad_args(xd, dyd, dw, g, ws=ws, target_blocks=4096, min_steps=2, atomic=2)
        for it in range(4):
            dw.fill_(float("nan"))
            hip._wgrad_full(a, ns, dw, hip.stream())
            torch.cuda.synchronize()
            err = ((dw.cpu() - dw_ref).norm() / dw_ref.norm()).item()
            nan = int(torch.isnan(dw).sum())
            tk = int(hip.wgrad_tickets.abs().sum())
            # the slabs as written by this launch, reduced by the separate kernel
            red = torch.empty_like(dw)
            hip.L.drn_splitk_reduce(a.out, red.data_ptr(), red.numel(), a.splits, 1.0, 0, hip.stream())
            torch.cuda.synchronize()
            err2 = ((red.cpu() - dw_ref).norm() / dw_ref.norm()).item()
            print(f"case {case} ns {ns} splits {a.splits} grid {hip.L.drn_wgrad_tiles(R*R*C, K)} it {it}: "
                  f"fused err {err:.3e} nan {nan} tickets {tk} | slabs->reduce err {err2:.3e}", flush=True)
