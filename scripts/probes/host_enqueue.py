#!/usr/bin/env python3
"""Host launch cost of one eager training step: with the GPU idle, time how long the host takes
to ENQUEUE a whole ResNet-50 step (forward + backward + SGD, ~320 kernel launches through the
ctypes backend) versus how long the GPU then takes to run it. Enqueue time well below the GPU
time means the eager step is GPU-bound (the host runs ahead); close to it means main-stream
gaps can come from the launch path.
usage: python scripts/probes/host_enqueue.py [--dataset imagenet] [--batch 128]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_resnet_tensorflow_amd.models.spec import build_spec
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="imagenet")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--cprofile", type=int, default=0, help="cProfile N steps, print the top host functions")
    a = ap.parse_args()
    spec = build_spec(a.dataset, 50)
    be = HipBackend("cuda")
    ex = Executor(spec, a.batch, be, "cuda", seed=1)
    be.synthetic_images(ex.images, seed=3)
    ex.labels.copy_(torch.randint(0, spec.num_classes, (a.batch,), dtype=torch.int32))
    ex.set_lr(0.1)
    ex.autotune()

    def step():
        ex.forward(train=True)
        ex.backward(defer_tail=True)
        ex.apply_gradients()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    for trial in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"trial {trial}: host enqueue {1e3 * (t1 - t0):.2f} ms, enqueue->done {1e3 * (t2 - t0):.2f} ms",
              flush=True)
    # steady state: back-to-back steps, host time per step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 20
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"steady: host {1e3 * (t1 - t0) / n:.2f} ms/step enqueued, wall {1e3 * (t2 - t0) / n:.2f} ms/step",
          flush=True)
    if a.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.cprofile):
            step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
