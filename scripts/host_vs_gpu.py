#!/usr/bin/env python3
"""Is the eager ResNet-50 step host-bound anywhere? For one eager step (bench setup: batch 128,
autotuned, high-priority main stream) record, at the start of the forward, of every backward
block and of the optimizer, the HOST time the enqueue reached that point and a GPU event on the
main stream. A point whose host time is later than its GPU time means the main stream ran dry
there, waiting for the host to launch.

usage: host_vs_gpu.py [batch]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.models.spec import build_spec  # noqa: E402
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend  # noqa: E402
from distributed_resnet_tensorflow_amd.parallel.engine import make_priority_stream  # noqa: E402
from distributed_resnet_tensorflow_amd.runtime.executor import Executor  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
be = HipBackend("cuda")
ex = Executor(build_spec("imagenet", 50), N, be, "cuda", seed=1234, weight_decay=1e-4)
be.synthetic_images(ex.images, seed=17)
ex.labels.copy_(torch.randint(0, 1001, (N,), dtype=torch.int32))
ex.set_lr(0.1)
ex.autotune()
prio = make_priority_stream()
marks = []


def mark(tag):
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    marks.append((tag, time.perf_counter(), ev))


orig = ex._block_bwd


def block_bwd(bp, bufs, cur):
    mark(f"bwd s{bp.blk.stage}b{bp.blk.index}")
    return orig(bp, bufs, cur)


ex._block_bwd = block_bwd


def step():
    mark("fwd")
    ex.forward(train=True)
    mark("bwd start")
    ex.backward(defer_tail=True)
    mark("sgd")
    ex.apply_gradients()
    mark("end")


with torch.cuda.stream(prio):
    for _ in range(5):
        marks.clear()
        step()
    torch.cuda.synchronize()
    marks.clear()
    t_sync = time.perf_counter()
    step()
    t_enq = time.perf_counter()
    torch.cuda.synchronize()
    t_done = time.perf_counter()
h0, e0 = marks[0][1], marks[0][2]
print(f"host enqueue of the step {1e3 * (t_enq - t_sync):.2f} ms, step wall {1e3 * (t_done - t_sync):.2f} ms")
print(f"{'point':14s} {'host ms':>8s} {'gpu ms':>8s} {'host lead ms':>12s}")
for tag, h, ev in marks:
    g = e0.elapsed_time(ev)
    print(f"{tag:14s} {1e3 * (h - h0):8.2f} {g:8.2f} {g - 1e3 * (h - h0):12.2f}")
