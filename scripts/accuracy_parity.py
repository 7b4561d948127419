#!/usr/bin/env python3
"""Training-accuracy parity on a learnable synthetic task (no dataset exists on these machines, so
the reference's CIFAR-10 top-1 -- README.md:19-30 of the reference -- cannot be reproduced; this
is the closest available evidence that the framework TRAINS like the reference's math).

Both runs start from the same initial weights (the executor's ParamStore, TF layouts) and see the
same batches:
  - drn: the product path -- HIP kernels, bf16 activations, fp32 master weights, hand-written
    backward, fused SGD-momentum (runtime/executor.py);
  - oracle: models/oracle.py, the pure-PyTorch fp32 autograd restatement of the reference's
    ResNet v2 (resnet_model_official.py) with torch.optim.SGD(momentum=0.9) and the reference's
    loss = cross-entropy + weight_decay * sum(l2 / 2) over all variables (measurement only).
Task: CIFAR-shaped 32x32x3 images, 10 classes; class c is a fixed smooth random template scaled by
a random contrast, circularly shifted by up to +-6 pixels, plus Gaussian pixel noise and a random
horizontal flip; every training step
draws a fresh batch (no memorisation), the test set is 2,560 held-out draws.

    python scripts/accuracy_parity.py [--depth 20] [--steps 400] [--noise 4.0]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from distributed_resnet_tensorflow_amd.models import oracle
from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor


def make_task(seed: int, noise: float):
    g = torch.Generator().manual_seed(seed)
    tmpl = F.interpolate(torch.randn(10, 3, 8, 8, generator=g), size=32, mode="bilinear", align_corners=False)
    tmpl = tmpl / tmpl.std(dim=(1, 2, 3), keepdim=True)

    def draw(n, gen):
        y = torch.randint(0, 10, (n,), generator=gen)
        a = 0.6 + 0.8 * torch.rand(n, 1, 1, 1, generator=gen)
        x = tmpl[y] * a
        sh = torch.randint(-6, 7, (n, 2), generator=gen)
        for i in range(n):  # random translation: a CNN's invariance, not a linear template match
            x[i] = x[i].roll((int(sh[i, 0]), int(sh[i, 1])), dims=(1, 2))
        x = x + noise * torch.randn(n, 3, 32, 32, generator=gen)
        flip = torch.rand(n, generator=gen) < 0.5
        x[flip] = x[flip].flip(-1)
        return x.permute(0, 2, 3, 1).contiguous(), y  # NHWC
    return draw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=20)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--wd", type=float, default=2e-4)
    ap.add_argument("--noise", type=float, default=4.0)
    ap.add_argument("--decay-at", type=float, default=0.75, help="fraction of the steps after which lr /= 10")
    ap.add_argument("--eval-every", type=int, default=250)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    N = a.batch
    spec = build_spec("cifar10", a.depth)
    draw = make_task(1, a.noise)
    gtest = torch.Generator().manual_seed(2)
    test = [draw(N, gtest) for _ in range(2560 // N)]

    ex = Executor(spec, N, HipBackend(), "cuda", seed=11, weight_decay=a.wd)
    p = {k: v.detach().float().cuda().requires_grad_(True) for k, v in oracle.params_from_store(ex.P, False).items()}
    st = {k: (m.cuda(), v.cuda()) for k, (m, v) in oracle.state_from_store(ex.P).items()}
    opt = torch.optim.SGD(list(p.values()), lr=a.lr, momentum=0.9)
    ex.set_lr(a.lr)

    def set_batch(x, y):
        ex.images.zero_()
        ex.images[..., :3] = x.cuda().bfloat16()
        ex.labels.copy_(y.to(torch.int32).cuda())

    def evaluate():
        cd = co = 0
        for x, y in test:
            set_batch(x, y)
            ex.forward(train=False)
            cd += int(ex.correct.sum())
            with torch.no_grad():
                logits = oracle.forward(spec, p, st, x.cuda(), training=False)
            co += int((logits.argmax(1).cpu() == y).sum())
        n = len(test) * N
        return cd / n, co / n

    gtrain = torch.Generator().manual_seed(3)
    curve = []
    for step in range(1, a.steps + 1):
        if step == int(a.decay_at * a.steps) + 1:  # the reference's piecewise-constant schedule, one drop
            ex.set_lr(a.lr / 10)
            for gr in opt.param_groups:
                gr["lr"] = a.lr / 10
        x, y = draw(N, gtrain)
        set_batch(x, y)
        ex.train_step()
        opt.zero_grad()
        _, xent, cost = oracle.loss_fn(spec, p, st, x.cuda(), y.cuda(), weight_decay=a.wd, training=True)
        cost.backward()
        opt.step()
        if step % 50 == 0 or step == 1:
            torch.cuda.synchronize()
            d_loss = float(ex.loss_vec.float().mean())
            acc = evaluate() if step % a.eval_every == 0 or step == a.steps else (None, None)
            row = {"step": step, "drn_xent": round(d_loss, 4), "oracle_xent": round(float(xent.detach()), 4),
                   "drn_test_top1": acc[0], "oracle_test_top1": acc[1]}
            curve.append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps({"final": True, "depth": a.depth, "noise": a.noise, "steps": a.steps,
                      "drn_test_top1": curve[-1]["drn_test_top1"],
                      "oracle_test_top1": curve[-1]["oracle_test_top1"]}), flush=True)
    if a.json:
        json.dump({"depth": a.depth, "steps": a.steps, "batch": N, "lr": a.lr, "wd": a.wd, "noise": a.noise,
                   "decay_at": a.decay_at, "curve": curve}, open(a.json, "w"))


if __name__ == "__main__":
    main()
