#!/usr/bin/env python3
"""Per-workgroup timeline of one LDS-DMA weight-gradient launch (drn_wgrad_trace_set): kernel span,
block lifetime split (prologue + main loop / partial-tile store), blocks resident per CU over time,
and the split-K reduction that follows, timed separately.
usage: trace_wgrad.py H C K R stride pipeline target [pro]
(needs the diagnostics build: python -m distributed_resnet_tensorflow_amd.ops.build --variant
 gpu_variants/trace -DDRN_CONV_TRACE, then DRN_KERNEL_LIB=gpu_variants/trace/libdrn_kernels.so)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend

H, C, K, R, st, ns, tgt = (int(v) for v in sys.argv[1:8])
flags = set(sys.argv[8:])
N = 128
be = HipBackend()
be.autotune = False
P = H // st
g = ConvGeom(st, (R - 1) // 2, (R - 1) // 2)
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
dw = torch.zeros(K, R, R, C, device="cuda")
in_bn = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1) if "pro" in flags else None
ws = torch.empty(max(16, be.wgrad_ws_elems(N * P * P, K, R, R, C)), device="cuda")
a = be.wgrad_args(x, dy, dw, g, in_bn=in_bn, ws=ws, target_blocks=tgt)
zp = be.zero_page.data_ptr()
stream = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    be._wgrad_full(a, ns, dw, stream)
torch.cuda.synchronize()
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
e0.record()
for _ in range(20):
    be._wgrad_kernel(a, ns, stream)
e1.record()
for _ in range(20):
    be._wgrad_full(a, ns, dw, stream)
e2.record()
torch.cuda.synchronize()
t_k = e0.elapsed_time(e1) / 20 * 1e3
t_f = e1.elapsed_time(e2) / 20 * 1e3
nblk = a.splits * be.L.drn_wgrad_tiles(R * R * C, K)
buf = torch.zeros(4 * (nblk + 64), dtype=torch.int64, device="cuda")
assert be.L.drn_wgrad_trace_set(buf.data_ptr()) == 0, "not a -DDRN_CONV_TRACE library"
torch.cuda.synchronize()
be._wgrad_kernel(a, ns, stream)
torch.cuda.synchronize()
be.L.drn_wgrad_trace_set(None)
tr = buf.view(-1, 4).cpu().numpy()
tr = tr[tr[:, 0] != 0]
t0 = tr[:, 0].min()
s, l, e = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0  # us
hw = tr[:, 3] & 0xffffffff
xcc = (tr[:, 3] >> 32) & 0xf
cuid = xcc * 64 + ((hw >> 13) & 0x7) * 16 + ((hw >> 12) & 1) * 8 + ((hw >> 8) & 0xf)
flops = 2.0 * N * P * P * K * R * R * C
print(f"H{H} C{C} K{K} R{R} s{st} pipe{ns} target{tgt} {sorted(flags)}: blocks {len(tr)} (splits {a.splits}, "
      f"{a.pix_per_split // 64} 64-px steps each)  kernel {t_k:.1f} us ({flops / t_k / 1e6:.0f} TF/s)  "
      f"kernel+reduce {t_f:.1f} us  traced span {e.max():.1f} us  distinct CUs {len(np.unique(cuid))}")
q = lambda v: f"mean {v.mean():6.2f} p10 {np.percentile(v, 10):6.2f} p50 {np.percentile(v, 50):6.2f} p90 {np.percentile(v, 90):6.2f}"
print(f"  lifetime  {q(e - s)}")
print(f"  main loop {q(l - s)}   per 64-px step {np.median(l - s) / max(1, a.pix_per_split // 64):.2f} us")
print(f"  store     {q(e - l)}")
ts = np.linspace(0, e.max(), 30)
res = [((s <= t) & (e > t)).sum() / max(1, len(np.unique(cuid))) for t in ts]
print("  resident blocks/CU over time: " + " ".join(f"{r:.1f}" for r in res))
hist, edges = np.histogram(s, bins=15)
print("  start histogram: " + " ".join(str(h) for h in hist) + f"  (bin {edges[1]:.1f} us)")
