#!/usr/bin/env python3
"""Per-operation time breakdown of one training step, in the real executor's call sequence.

Every HipBackend kernel call of the step is bracketed by device events on ONE stream (the
weight-gradient side stream is disabled so the calls serialise), labelled by op, tensor shape
and fused-epilogue flags, and aggregated by label. The sum is the serialized busy time (the real
step overlaps the weight gradients with the data-gradient chain).
usage: python scripts/op_breakdown.py [--dataset imagenet] [--batch 128] [--steps 3] [--top 60]
"""
import argparse
import collections
import os
import sys

os.environ["DRN_WGRAD_STREAM"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor

OPS = ["conv_fwd", "conv_wgrad", "bn_stats", "bn_finalize", "bn_apply", "bn_bwd_reduce", "bn_finalize_bwd",
       "bn_apply_fin", "bn_bwd_apply_fin",
       "bn_bwd_apply", "bn_apply_stats", "bn_bwd_apply_stats", "pool_bnrelu", "sgemm", "softmax_xent", "colsum",
       "maxpool_fwd", "maxpool_bwd", "sgd_momentum", "cast_bf16", "weight_tflip", "zero_"]


def shp(t):
    return "x".join(str(d) for d in t.shape) if isinstance(t, torch.Tensor) else "-"


def label(op, args, kw):
    if op == "conv_fwd":
        x, w, y, g = args[:4]
        flags = [k for k in ("in_bn", "residual", "stats", "out_map", "bn_bwd", "bn_fin", "in_fin")
                 if kw.get(k) is not None]
        if kw.get("out_fill"):
            flags.append("fill")
        kind = "dgrad" if (kw.get("bn_bwd") is not None or kw.get("out_map") is not None or
                           w.shape[0] == x.shape[-1] and w.shape[-1] != x.shape[-1]) else "conv"
        return f"{kind} x{shp(x)} w{shp(w)} s{g.stride} {'+'.join(flags)}"
    if op == "conv_wgrad":
        x, dy = args[:2]
        return f"wgrad x{shp(x)} dy{shp(dy)} {'pro' if kw.get('in_bn') is not None else ''}"
    t = next((a for a in args if isinstance(a, torch.Tensor)), None)
    return f"{op} {shp(t)}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="imagenet")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=70)
    a = ap.parse_args()
    spec = build_spec(a.dataset, a.resnet_size)
    be = HipBackend("cuda")
    ex = Executor(spec, a.batch, be, "cuda", seed=1, weight_decay=1e-4)
    be.synthetic_images(ex.images, seed=3)
    ex.labels.copy_(torch.randint(0, spec.num_classes, (a.batch,), dtype=torch.int32))
    ex.set_lr(0.1)
    ex.autotune()
    rec = []
    on = [False]
    for op in OPS:
        fn = getattr(be, op, None)
        if fn is None:
            continue

        def wrap(*args, _fn=fn, _op=op, **kw):
            if not on[0]:
                return _fn(*args, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = _fn(*args, **kw)
            e.record()
            rec.append((label(_op, args, kw), s, e))
            return r
        setattr(be, op, wrap)
    for i in range(a.steps + 1):
        on[0] = i == a.steps
        ex.train_step()
    torch.cuda.synchronize()
    agg = collections.OrderedDict()
    for lab, s, e in rec:
        t = s.elapsed_time(e) * 1e3
        n, tot = agg.get(lab, (0, 0.0))
        agg[lab] = (n + 1, tot + t)
    total = sum(t for _, t in agg.values())
    print(f"serialized busy {total:.1f} us over {len(rec)} calls")
    fam = collections.defaultdict(float)
    for lab, (n, t) in agg.items():
        fam[lab.split()[0]] += t
    print("--- by op ---")
    for k, t in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"{t:9.1f} us  {100 * t / total:5.1f}%  {k}")
    print("--- by label ---")
    for lab, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{t:9.1f} us  n={n:2d}  {t / n:7.1f} us/call  {lab}")


if __name__ == "__main__":
    main()
