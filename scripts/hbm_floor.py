#!/usr/bin/env python3
"""Compulsory HBM bytes of one training step, per backend op (the floor the PMC-measured bytes of
scripts/pmc_report.py are compared against).

Runs one eager ResNet-50 step (bench configuration) with every HipBackend op wrapped: an op's
compulsory bytes = the sizes of the distinct tensors it touches (inputs read once, outputs written
once; a tensor that is both -- in-place applies, accumulating data gradients -- counted twice).
Re-reads a kernel makes beyond that (operand tiles fetched once per output tile, split-K partials,
statistics atomics) are what the measured bytes add on top.

    python scripts/hbm_floor.py [--batch 128] [--out floor.json]
"""
import argparse
import collections
import dataclasses
import json

import torch

from distributed_resnet_tensorflow_amd.models.spec import imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor

OPS = ("conv_fwd", "conv_wgrad", "bn_", "maxpool_", "sgemm", "colsum", "softmax_xent", "pool_bnrelu",
       "sgd_momentum", "weight_tflip", "stem_", "zero_", "fill_")


def _tensors(v, out):
    if isinstance(v, torch.Tensor):
        out.append(v)
    elif isinstance(v, (tuple, list)):
        for x in v:
            _tensors(x, out)
    elif dataclasses.is_dataclass(v) and not isinstance(v, type):
        for f in dataclasses.fields(v):
            _tensors(getattr(v, f.name), out)


def op_bytes(args, kwargs) -> int:
    ts = []
    _tensors(list(args) + list(kwargs.values()), ts)
    seen = collections.Counter()
    size = {}
    for t in ts:
        if t.numel() == 0:
            continue
        k = (t.data_ptr(), t.numel() * t.element_size())
        seen[k] += 1
        size[k] = k[1]
    return sum(size[k] * min(n, 2) for k, n in seen.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    be = HipBackend("cuda")
    ex = Executor(imagenet_resnet_v2(50), a.batch, be, "cuda", seed=1)
    be.synthetic_images(ex.images, seed=1)
    ex.autotune()
    for _ in range(2):
        ex.train_step(lr=0.01)
    torch.cuda.synchronize()
    rec = []
    for name in dir(be):
        if name.startswith("_") or not name.startswith(OPS):
            continue
        f = getattr(be, name)
        if not callable(f):
            continue

        def wrap(f=f, name=name):
            def g(*args, **kw):
                if depth[0] == 0:   # outermost op only (composite ops call other ops)
                    rec.append((name, op_bytes(args, kw)))
                depth[0] += 1
                try:
                    return f(*args, **kw)
                finally:
                    depth[0] -= 1
            return g
        setattr(be, name, wrap())
    depth = [0]
    ex.train_step(lr=0.01)
    torch.cuda.synchronize()
    by = collections.defaultdict(lambda: [0, 0])
    for n, b in rec:
        by[n][0] += 1
        by[n][1] += b
    total = sum(v[1] for v in by.values())
    res = {n: {"calls": c, "MB": round(b / 1e6, 1)} for n, (c, b) in sorted(by.items(), key=lambda kv: -kv[1][1])}
    print(f"{'op':24s} {'calls':>5s} {'floor MB':>9s}")
    for n, v in res.items():
        print(f"{n:24s} {v['calls']:5d} {v['MB']:9.1f}")
    print(f"total compulsory {total / 1e9:.2f} GB per step")
    if a.out:
        json.dump({"batch": a.batch, "ops": res, "total_GB": round(total / 1e9, 3)}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
