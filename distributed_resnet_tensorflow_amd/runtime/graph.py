"""HIP-graph capture of a whole training step.

CIFAR-size steps are ~500 kernel launches of a few microseconds each, so host launch cost would
dominate. The executor issues every launch on the current stream with raw
device pointers into pre-allocated buffers and reads the learning rate from device memory, so the
complete forward + backward (+ all-reduce) + SGD sequence is captured once with
``torch.cuda.CUDAGraph`` (= hipGraph on ROCm) and replayed per step.
"""
from __future__ import annotations

from typing import Callable

import torch


class StepGraph:
    def __init__(self, step_fn: Callable[[], None], warmup: int = 2, pool=None):
        self.step_fn = step_fn
        self.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):  # first launches set kernel attributes outside capture
                step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(self.graph, pool=pool):
            step_fn()
        torch.cuda.synchronize()

    def replay(self):
        self.graph.replay()
