#!/usr/bin/env python3
"""Per-workgroup timeline of one LDS-DMA conv launch (drn_conv_trace_set): kernel span, block
lifetime split (prologue+main loop / epilogue), blocks resident per CU over time.
usage: trace_conv.py H C K R stride cfg [flags: pro res stats]
(needs the diagnostics build: DRN_CONV_TRACE=1 python -m distributed_resnet_tensorflow_amd.ops.build)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend

H, C, K, R, st, cfg = (int(v) for v in sys.argv[1:7])
flags = set(sys.argv[7:])
N = 128
be = HipBackend()
be.autotune = False
be.forced_cfg = cfg
P = H // st
g = ConvGeom(st, (R - 1) // 2, (R - 1) // 2)
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
kw = {}
if "pro" in flags:
    kw["in_bn"] = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1)
if "res" in flags:
    kw["residual"] = torch.randn_like(y)
if "stats" in flags:
    kw["stats"] = torch.zeros(8, 2, K, device="cuda")
for _ in range(5):
    be.conv_fwd(x, w, y, g, **kw)
buf = torch.zeros(4 * 200000, dtype=torch.int64, device="cuda")
be.L.drn_conv_trace_set(buf.data_ptr())
torch.cuda.synchronize()
be.conv_fwd(x, w, y, g, **kw)
torch.cuda.synchronize()
be.L.drn_conv_trace_set(None)
tr = buf.view(-1, 4).cpu().numpy()
tr = tr[tr[:, 0] != 0]
t0 = tr[:, 0].min()
s, l, e = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0  # us
hw = tr[:, 3] & 0xffffffff
xcc = (tr[:, 3] >> 32) & 0xf
cu = (hw >> 8) & 0xf
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
cuid = xcc * 64 + se * 16 + sh * 8 + cu  # unique-ish CU key
print(f"H{H} C{C} K{K} R{R} s{st} cfg{cfg} {sorted(flags)}: blocks {len(tr)}  span {e.max():.1f} us  "
      f"distinct CUs {len(np.unique(cuid))}")
life, loop, epi = e - s, l - s, e - l
q = lambda v: f"mean {v.mean():6.2f} p10 {np.percentile(v, 10):6.2f} p50 {np.percentile(v, 50):6.2f} p90 {np.percentile(v, 90):6.2f}"
print(f"  lifetime  {q(life)}")
print(f"  main loop {q(loop)}")
print(f"  epilogue  {q(epi)}")
# concurrency: blocks resident per CU, sampled
ts = np.linspace(0, e.max(), 40)
res = [((s <= t) & (e > t)).sum() / max(1, len(np.unique(cuid))) for t in ts]
print("  resident blocks/CU over time: " + " ".join(f"{r:.1f}" for r in res))
# start-time histogram (rounds)
hist, edges = np.histogram(s, bins=20)
print("  start histogram: " + " ".join(str(h) for h in hist) + f"  (bin {edges[1]:.1f} us)")
bidx = np.nonzero(buf.view(-1, 4).cpu().numpy()[:, 0])[0]
match = float(np.mean((bidx % 8) == xcc))
print(f"  blocks whose XCC == blockIdx % 8: {match * 100:.1f}%   XCC histogram: {np.bincount(xcc, minlength=8).tolist()}")
