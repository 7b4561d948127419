"""Native step launcher: one eager training step recorded once, replayed from C++.

The eager step (runtime/executor.py) is ~340 kernel launches (ResNet-50) on the critical-path
stream and the weight-gradient side stream, ordered by cross-stream events. Issued from Python it
costs the host ~19 us per launch (6.4 ms per ResNet-50 step, more than the GPU time of a CIFAR
step); a HIP graph removes that cost but replays every branch from one normal-priority queue and
measured slower for ResNet-50 (10.4 vs 9.6 ms, profiles/r4_graph_vs_eager_ab.txt).

A StepPlan records the executor's step through the kernel library's recording mode
(csrc/kernels/plan.hip: every `drn::launch` of the calling thread appends {kernel, grid, block,
LDS, stream, argument copy}) while the executor's stream ordering goes through a PlanSched (event
record / stream wait entries instead of torch's stream API). `replay()` re-issues the entries with
`drn_plan_replay` -- the same kernels, arguments, streams and priorities as the eager step, one
host call per segment. Data-parallel steps over RCCL are cut where the eager step hands a bucket
to the engine: at replay, each cut runs the engine's Python side (begin_step, the bucket
collectives issued from the report stream, finish) between two native segments. With the P2P
all-reduce (parallel/p2p.py) every collective is a library kernel synchronised by device-side
epoch flags, so the step boundary, the bf16 wire casts, the bucket reductions on the P2P comm
stream and their cross-stream ordering are recorded too: the data-parallel step is ONE native
segment (the CIFAR 4-GPU configuration; before, P2P steps could only be one HIP graph).

The reference's counterpart is the TF1 C++ executor running the captured train_op every
`mon_sess.run` (resnet_cifar_main.py:320-321).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch

from ..ops import _lib


class TorchSched:
    """Cross-stream ordering through torch's stream / event API (eager steps, graph capture)."""
    recording = False

    def record(self, stream, key: Optional[str] = None):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def wait(self, stream, ev, key: Optional[str] = None):
        stream.wait_event(ev)

    def wait_stream(self, dst, src):
        dst.wait_stream(src)

    def done(self, ev) -> bool:
        return ev.query()


class _PlanEvent:
    __slots__ = ("idx",)

    def __init__(self, idx: int):
        self.idx = idx


class PlanSched:
    """Cross-stream ordering recorded into a native plan. `key`ed events are the ones a step
    waits on at its start and records at its end (the data-gradient weight refresh): the wait
    of replay k then refers to the record of replay k-1, as the eager steps' events do."""
    recording = True

    def __init__(self, plan: "StepPlan"):
        self.plan = plan
        self.keyed = {}
        self.waited_keys, self.recorded_keys = set(), set()

    def _new(self) -> int:
        i = self.plan.L.drn_plan_new_event(self.plan.p)
        if i < 0:
            raise _lib.KernelLibraryError(f"drn_plan_new_event failed with hipError {-i}")
        return i

    def _idx(self, key: Optional[str]) -> int:
        if key is None:
            return self._new()
        if key not in self.keyed:
            self.keyed[key] = self._new()
        return self.keyed[key]

    def record(self, stream, key: Optional[str] = None):
        i = self._idx(key)
        if key is not None:
            self.recorded_keys.add(key)
        _lib.check(self.plan.L.drn_plan_event_record(self.plan.p, i, ctypes.c_void_p(stream.cuda_stream)),
                   "drn_plan_event_record")
        return _PlanEvent(i)

    def wait(self, stream, ev, key: Optional[str] = None):
        if isinstance(ev, _PlanEvent):
            i = ev.idx
        elif key is not None:           # an event of the previous (eager) step: the keyed slot
            i = self._idx(key)
            self.waited_keys.add(key)
        else:
            raise RuntimeError("a native plan may only wait on its own events or keyed carry-in events")
        _lib.check(self.plan.L.drn_plan_stream_wait(self.plan.p, ctypes.c_void_p(stream.cuda_stream), i),
                   "drn_plan_stream_wait")

    def wait_stream(self, dst, src):
        self.wait(dst, self.record(src))

    def done(self, ev) -> bool:
        return False                    # replay-time completion is unknown: always order

    def cut(self, action):
        self.plan._cut(action)


class StepPlan:
    """One training step of `ex` (single GPU: forward, backward with the deferred stem tail,
    update; with `engine`: forward, begin_step, backward cut at every bucket report, finish,
    update) recorded after one eager warm-up step, replayed natively. The caller keeps the
    stream context it recorded under (the recorded launches name their streams explicitly)."""

    def __init__(self, ex, engine=None, grad_scale: float = 1.0, warmup: int = 1, threads: int = 1):
        self.L = _lib.lib()
        self.ex, self.eng, self.grad_scale = ex, engine, grad_scale
        if engine is not None and (engine.mode != "sync" or engine.zero1):
            raise ValueError("native plans cover the synchronous, unsharded data-parallel engine")
        self.p2p = engine.p2p if engine is not None else None
        for _ in range(warmup):         # kernel attributes, workspaces, tuning: all outside the plan
            self._eager()
        torch.cuda.synchronize()
        self.p = ctypes.c_void_p(self.L.drn_plan_create())
        self.cuts: List[Tuple[int, object]] = []
        self._grad = None
        be = ex.be
        sched, old = PlanSched(self), ex.sched
        ex.sched, be.recording = sched, True
        if self.p2p is not None:
            sched.native_reports = True       # (the executor issues the bucket kernels while recording)
            self.p2p.sched = sched
        elif engine is not None:
            ex.grad_ready = lambda lo: None   # (reports become plan cuts: PlanSched.cut)
        _lib.check(self.L.drn_plan_record_begin(self.p), "drn_plan_record_begin")
        ok = False
        try:
            ex.forward(train=True)
            if engine is None:
                ex.backward(defer_tail=not ex.check_nan)
                ex.apply_gradients()
            elif self.p2p is not None:
                engine.begin_step()
                ex.backward()
                self._grad = engine.finish()
                engine.apply_gradients(self._grad, grad_scale)
            else:
                self._cut("begin")
                ex.backward()
                self._cut("finish")
                self._grad = engine.wire_buf if engine.wire_buf is not None else ex.P.grad
                ex.apply_gradients(grad_scale=grad_scale, grad=self._grad)
            ok = True
        finally:
            self.L.drn_plan_record_end()
            ex.sched, be.recording = old, False
            ex.grad_ready = None
            if self.p2p is not None:
                self.p2p.sched = None
            if not ok:
                # a failed recording leaves plan events in the executor's carry-over state: the
                # next eager step would hand them to torch's stream API
                self._clear_carry()
        self._cut(None)
        if sched.recorded_keys != sched.waited_keys:
            raise RuntimeError(f"plan carry-in events unbalanced: recorded {sched.recorded_keys}, "
                               f"waited {sched.waited_keys} (record the plan after an eager step)")
        # the recorded step's events are plan events: an eager step after replays must not wait on
        # them through torch; replay() leaves a torch event for the side-stream weight refresh
        self._clear_carry()
        self._tflip = "tflip" in sched.recorded_keys
        self._tflip_torch = None
        self.launches = int(self.L.drn_plan_launches(self.p))
        self.set_threads(threads)
        torch.cuda.synchronize()

    def _clear_carry(self):
        ex = self.ex
        ex._tflip_ev = ex._tail_ev = ex._stem_ev = None
        ex._marks.clear()
        ex._pending.clear()

    def set_threads(self, n: int):
        """Host threads issuing a replay: 1 = the calling thread, in recorded order; n > 1 = one
        thread per stream (the critical-path and weight-gradient streams' launches enqueued
        concurrently, cross-stream events in recorded order; csrc/kernels/plan.hip)."""
        _lib.check(self.L.drn_plan_set_threads(self.p, int(n)), "drn_plan_set_threads")
        self.threads = int(n)

    def stats(self) -> dict:
        L, p = self.L, self.p
        return {"launches": self.launches, "event_records": int(L.drn_plan_count(p, 1)),
                "live_event_records": int(L.drn_plan_live_records(p)),
                "stream_waits": int(L.drn_plan_count(p, 2)), "streams": int(L.drn_plan_lanes(p)),
                "segments": sum(1 for _, a in self.cuts if a is not None) + 1, "threads": self.threads}

    def _eager(self):
        ex, eng = self.ex, self.eng
        ex.forward(train=True)
        if eng is None:
            ex.backward(defer_tail=not ex.check_nan)
            ex.apply_gradients()
        else:
            eng.begin_step()
            ex.backward()
            eng.apply_gradients(eng.finish(), self.grad_scale)

    def _cut(self, action):
        self.cuts.append((int(self.L.drn_plan_size(self.p)), action))

    def replay(self):
        L, p, ex, eng = self.L, self.p, self.ex, self.eng
        if self.p2p is not None:
            # one segment; the host side of the step is the engine's replay bookkeeping and the
            # error word's copy into pinned memory (P2PAllReduce.end_step, eager)
            eng.replay_begin()
            _lib.check(L.drn_plan_replay(p, 0, self.cuts[-1][0]), "drn_plan_replay")
            self.p2p.err_host.copy_(self.p2p.err, non_blocking=True)
            eng.replay_end()
            self._after_replay()
            return
        begin = 0
        for end, action in self.cuts:
            if end > begin:
                _lib.check(L.drn_plan_replay(p, begin, end), "drn_plan_replay")
            begin = end
            if action is None:
                continue
            if action == "begin":
                eng.begin_step()
            elif action == "finish":
                g = eng.finish()
                assert g is self._grad, "the recorded update reads a different gradient buffer"
            else:                       # ("report", lo): the bucket collectives, live
                ex._report(action[1])
        self._after_replay()

    def _after_replay(self):
        ex = self.ex
        if self.eng is None:
            ex._tail_ev = None          # (the recorded step joined its deferred tail itself)
        if self._tflip and ex.side is not None:
            # the replay ended with the data-gradient weight refresh on the side stream: an eager
            # backward after it waits for that refresh (a torch event after the side stream's
            # replayed work, as the eager step's own "tflip" event would be)
            if self._tflip_torch is None:
                self._tflip_torch = torch.cuda.Event()
            self._tflip_torch.record(ex.side)
            ex._tflip_ev = self._tflip_torch

    def close(self):
        if self.p is not None:
            self.L.drn_plan_destroy(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass
