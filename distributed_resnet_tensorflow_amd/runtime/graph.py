"""HIP-graph capture of a whole training step.

CIFAR-size steps are ~500 kernel launches of a few microseconds each, so host launch cost would
dominate. The executor issues every launch on the current stream with raw
device pointers into pre-allocated buffers and reads the learning rate from device memory, so the
complete forward + backward (+ all-reduce) + SGD sequence is captured once with
``torch.cuda.CUDAGraph`` (= hipGraph on ROCm) and replayed per step. Data-parallel steps whose
collectives are host-issued RCCL calls use a chain of per-segment graphs instead
(SegmentedStepGraph).
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


class SegmentedStepGraph:
    """Data-parallel step as a chain of HIP graphs with the gradient collectives between them.

    RCCL collectives are issued from the host (`torch.distributed`), so instead of capturing
    them the step is cut at the executor's gradient-ready points: graph i ends at the i-th
    `grad_ready(lo)` report of the backward (graph 0 also holds the forward), the last graph is
    the fused SGD update. Replay launches each graph and then hands its `lo` to the engine, which
    fires every bucket that became complete on RCCL's stream -- the same overlap as the eager
    path, at ~20 graph launches per step instead of ~450 kernel launches (eager ImageNet
    ResNet-50 is host-bound).
    All buffers are preallocated by the executor, so no capture allocates.
    """

    def __init__(self, ex, engine, grad_scale: float, warmup: int = 1):
        if engine.p2p is not None or engine.mode != "sync" or engine.zero1:
            # (ZeRO-1 updates per-rank shards and all-gathers the weights: not one captured SGD)
            raise ValueError("segmented graphs are for the synchronous, unsharded RCCL/gloo engine")
        self.ex, self.eng, self.grad_scale = ex, engine, grad_scale
        # a capture may end only when every forked stream has joined: the side-stream weight
        # gradients (reported one block late) would straddle the cut points, so this step keeps
        # them on the main stream
        self._side, ex.side = ex.side, None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.segments = []   # (graph, lo reported after it); the last graph runs after finish()
        self._g = None
        with torch.cuda.stream(s):
            self._open()
            ex.forward(train=True)
            ex.grad_ready = self._cut       # backward ends with grad_ready(0): the open graph
            try:                            # then holds only the SGD update
                ex.backward()
            finally:
                ex.grad_ready = None
            # the SGD segment reads the buffer finish() returns: with the bf16 wire that is the
            # reduced bf16 shadow, never the rank-local fp32 gradient
            ex.apply_gradients(grad_scale=grad_scale, grad=self._reduced_grad())
            self._close(None)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    @property
    def side_stream(self):
        """The executor's weight-gradient side stream this graph took off it (an eager step
        that replaces the graph puts it back)."""
        return self._side

    def _reduced_grad(self):
        return self.eng.wire_buf if self.eng.wire_buf is not None else self.ex.P.grad

    def _eager(self):
        ex, eng = self.ex, self.eng
        ex.forward(train=True)
        eng.begin_step()
        ex.backward()
        g = eng.finish()
        ex.apply_gradients(grad_scale=self.grad_scale, grad=g)

    def _open(self):
        self._g = torch.cuda.CUDAGraph()
        self._g.capture_begin()

    def _close(self, lo):
        self._g.capture_end()
        self.segments.append((self._g, lo))
        self._g = None

    def _cut(self, lo: int):
        self._close(lo)
        self._open()

    def replay(self):
        eng = self.eng
        eng.begin_step()
        eng.ex.grad_ready = None          # the recorded cut points stand in for the hook
        for g, lo in self.segments[:-1]:
            g.replay()
            eng._on_ready(lo)
        g = eng.finish()
        assert g is self._reduced_grad(), "the captured SGD segment reads a different gradient buffer"
        self.segments[-1][0].replay()
