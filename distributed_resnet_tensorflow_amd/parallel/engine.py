"""Data-parallel engine: bucketed gradient all-reduce overlapped with the backward pass.

Replaces both distribution strategies of the reference:
  * SyncReplicasOptimizer over parameter servers (resnet_model.py:101-112, CS1-CS3): every
    worker pushes gradients to PS accumulators, the chief averages N of them and applies
    Momentum. Mathematically that is "average the N replicas' gradients, then every replica
    applies the same update" -- which is exactly an all-reduce(mean) + identical local SGD, with
    no PS process and no per-step variable fetch.
  * Horovod DistributedOptimizer (resnet_model.py:114-116) + BroadcastGlobalVariablesHook(0)
    (resnet_cifar_main_horovod.py:316): same all-reduce, plus a rank-0 broadcast at start.

MI355X design: one process per GPU, torch.distributed "nccl" (= RCCL over xGMI). The flat
gradient buffer (runtime/params.py) is cut into contiguous buckets in REVERSE creation order;
the executor reports, after every residual block's backward, the lowest flat offset whose
gradients are complete, and every bucket that is fully complete is all-reduced immediately
(async op on RCCL's stream, ordered after the producing kernels) while earlier blocks are still
back-propagating. `finish()` makes the compute stream wait for the last bucket before the
fused SGD launch. The average's 1/N is folded into the SGD kernel (grad_scale). Bucket sizes
grow from 2 MB at the start of the buffer (stem / stage 1, produced last) to the 25 MB cap:
ResNet-50's 102 MB of fp32 gradients -> 3 large buckets that run RCCL at link bandwidth on the
7 point-to-point xGMI links while the backward pass continues, and small final buckets, so only
~2 MB of all-reduce is left exposed after the backward pass.

Parameter sharding over PS tasks maps to the optional ZeRO-1 mode
(`shard_optimizer=True`, --optimizer_sharding): buckets are cut at multiples of 64 * world
elements and REDUCE-SCATTERED instead of all-reduced, each rank runs the fused SGD-momentum on
its 1/world slice of every bucket (so momentum updates and optimizer HBM traffic are sharded),
then the bf16 compute weights are ALL-GATHERED (half the bytes of fp32): per step 0.75x the
collective bytes of the all-reduce path, with the weight gather exposed after the backward pass.
Masters / momentum outside a rank's shard go stale and are all-gathered by `gather_state()`
before a checkpoint is written (a collective: every rank takes part in the save decision).

Async PS training (--sync_replicas=False with --job_name set) maps to
`mode="delayed"`: step t applies the averaged gradient of step t-1 while step t's all-reduce
runs behind step t+1's compute (bounded staleness 1, no PS).
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from .watchdog import CollectiveWatchdog


def use_priority_main_stream():
    """Run this thread's subsequent GPU work (the eager data-parallel step) on a HIGH-priority
    stream. HIP serves each priority level from its own hardware queues; with the default 4 HW
    queues per process, once RCCL's streams exist a normal-priority main stream was measured
    sharing one in-order queue with the executor's weight-gradient side stream -- no
    wgrad/dgrad overlap (one-GPU single-rank engine: 12.9-13.0 ms vs 11.3 ms per ResNet-50 step).
    Not for HIP-graph capture: a graph replayed from a high-priority stream measured 19.4 vs
    11.2 ms. Returns the stream (None without a GPU)."""
    s = make_priority_stream()
    if s is not None:
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(s)
    return s


def make_priority_stream():
    """The high-priority stream use_priority_main_stream() switches to, without switching: for a
    caller that runs only its eager steps on it (bench.py's auto mode, whose HIP-graph candidate
    must stay on a normal-priority stream). None when there is no GPU."""
    if not torch.cuda.is_available():
        return None
    return torch.cuda.Stream(priority=-1)


def p2p_wanted(allreduce: str, grad_bytes: int, world: int, mode: str = "sync", shard_optimizer: bool = False,
               p2p_max_mb: float = 64.0) -> bool:
    """The one decision of whether the data-parallel step uses the P2P all-reduce (shared by the
    engine and bench.py). `p2p` forces it (the engine then validates the combination); `auto`
    picks it only for a small whole gradient (latency-bound CIFAR buckets) on ONE node
    (LOCAL_WORLD_SIZE == WORLD_SIZE: HIP IPC cannot map a peer on another host), synchronous
    mode and no optimizer sharding (which needs reduce-scatter / all-gather collectives)."""
    if allreduce == "p2p":
        return True
    if allreduce != "auto" or world > 8 or mode != "sync" or shard_optimizer:
        return False
    if int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) != world:
        return False
    return grad_bytes <= p2p_max_mb * (1 << 20)


def all_ranks_on_one_host(group=None) -> bool:
    """Whether every rank of `group` runs on this host (a collective: every rank must call it).
    HIP IPC maps peer buffers only within one node; the launch environment's LOCAL_WORLD_SIZE is
    set by torchrun and parallel/launch.py but not by --worker_hosts or MPI launches, so the P2P
    choice is confirmed against the ranks' host identities instead of trusting it."""
    import socket
    if dist.get_world_size(group) == 1:
        return True
    ident = socket.gethostname()
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            ident += "/" + f.read().strip()
    except OSError:
        pass
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, ident, group=group)
    return len(set(names)) == 1


class DataParallelEngine:
    def __init__(self, executor, bucket_mb: float = 25.0, mode: str = "sync", group=None,
                 allreduce: str = "rccl", p2p_max_mb: float = 64.0, first_bucket_mb: float = 2.0,
                 timeout_s: float = 0.0, shard_optimizer: bool = False, wire: str = ""):
        self.ex = executor
        self.P = executor.P
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.mode = mode
        self.buckets = self._make_buckets(int(bucket_mb * (1 << 20) // 4), int(first_bucket_mb * (1 << 20) // 4))
        # --allreduce: rccl | p2p (one-shot HIP IPC kernel, parallel/p2p.py) | auto (p2p when the
        # whole gradient is small -- latency-bound CIFAR buckets -- and the job is one GPU node)
        self.p2p = None
        # gradient dtype on the wire (--allreduce_wire / DRN_ALLREDUCE_WIRE): fp32, or bf16 (half
        # the collective bytes; fp32 master gradients, like Horovod's fp16 compression)
        self.wire = (wire or os.environ.get("DRN_ALLREDUCE_WIRE", "fp32")).lower()
        if self.wire not in ("fp32", "bf16"):
            raise ValueError(f"all-reduce wire type must be fp32 or bf16, got {self.wire!r}")
        want = p2p_wanted(allreduce, self.P.total * 4, self.world, mode, shard_optimizer, p2p_max_mb)
        if want and allreduce == "auto" and not all_ranks_on_one_host(group):
            want = False  # (--allreduce=p2p across hosts is refused by the IPC mapping itself)
        if want and self.P.grad.is_cuda and mode == "sync" and self.world <= 8 \
                and dist.get_backend(group) in ("nccl", "gloo"):
            from .p2p import P2PAllReduce
            if len(self.buckets) + 1 >= 64:
                self.buckets = self._make_buckets(int(self.P.total // 60) + 1)
            self.p2p = P2PAllReduce(self.P.grad, group, wire=self.wire)
        self.zero1 = bool(shard_optimizer) and self.world > 1 and mode == "sync"
        if self.zero1 and self.wire != "fp32":
            raise ValueError("optimizer sharding reduce-scatters fp32 gradients (--allreduce_wire=fp32)")
        # RCCL bf16 wire: a bf16 shadow of the flat gradient; each bucket is cast into it by an
        # in-tree kernel on the compute stream and all-reduced THERE, and the fused SGD reads the
        # reduced bf16 buffer directly (no cast-back pass). The sum is accumulated in bf16 inside
        # RCCL (rounding grows with the rank count; the P2P bf16 wire accumulates in fp32)
        self.wire_buf = None
        if self.wire == "bf16" and self.p2p is None and mode == "sync":
            self.wire_buf = torch.zeros(self.P.total, dtype=torch.bfloat16, device=self.P.grad.device)
        if self.zero1:
            if self.p2p is not None:
                raise ValueError("optimizer sharding uses reduce-scatter / all-gather collectives, not --allreduce=p2p")
            self.buckets = self._align_buckets(self.buckets, 64 * self.world)
        self.works: List = []
        self.launched = [False] * len(self.buckets)
        self.frontier = self.P.total
        self._delayed_pending = False
        if mode == "delayed":
            self.comm_grad = torch.zeros_like(self.P.grad)
            self.ready_grad = torch.zeros_like(self.P.grad)
        # observability: per-step backward time, all-reduce time left exposed after
        # the backward pass, and the overlap fraction; device events on GPU, host clock on CPU
        self.cuda = self.P.grad.is_cuda
        self._ev = None
        self._host_t = None
        self._step_no = 0
        self.watchdog = CollectiveWatchdog(timeout_s, rank=self.rank) if timeout_s > 0 else None

    # -- bucket layout ---------------------------------------------------------------------------
    def _make_buckets(self, cap_elems: int, first_elems: int = 0):
        """Contiguous [lo, hi) slices cut at slot boundaries, returned in the order they become
        ready (end of the flat buffer first). Sizes grow geometrically from the START of the
        buffer (the stem / first stage, whose gradients are produced last): first_elems, 2x, 4x,
        ... capped at cap_elems, so the bucket left exposed after the backward pass is small
        while the early (large-layer) buckets stay large enough for link-bandwidth RCCL."""
        bounds = [s.offset for s in self.P.slots] + [self.P.total]
        first_elems = min(first_elems or cap_elems, cap_elems)
        buckets, lo, want = [], 0, first_elems
        for b in bounds[1:]:
            if b - lo >= want:
                buckets.append((lo, b))
                lo, want = b, min(2 * want, cap_elems)
        if lo < self.P.total:
            buckets.append((lo, self.P.total))
        return buckets[::-1]

    def _align_buckets(self, buckets, align: int):
        """Bucket boundaries rounded down to multiples of `align` (= 64 * world), so every bucket
        but the one ending at the buffer's end splits into `world` equal 256-byte-aligned shards.
        A bucket is still launched only once its whole range is complete (lo >= frontier)."""
        bounds = sorted({(lo // align) * align for lo, _ in buckets} | {0})
        out, prev = [], None
        for b in bounds + [self.P.total]:
            if prev is not None and b > prev:
                out.append((prev, b))
            prev = b
        return out[::-1]

    def _sharded(self, lo: int, hi: int) -> bool:
        return self.zero1 and (hi - lo) % self.world == 0

    def _shard(self, lo: int, hi: int):
        """This rank's slice of bucket [lo, hi) (the whole bucket when it is not sharded)."""
        if not self._sharded(lo, hi):
            return lo, hi
        c = (hi - lo) // self.world
        return lo + self.rank * c, lo + (self.rank + 1) * c

    # -- hooks --------------------------------------------------------------------------------------
    def begin_step(self):
        self.works = []
        self.launched = [False] * len(self.buckets)
        self.frontier = self.P.total
        self._step_no += 1
        if self.watchdog is not None:
            self.watchdog.arm(self._step_no)
        if self.cuda and (torch.cuda.is_current_stream_capturing() or getattr(self.ex.sched, "recording", False)):
            self._ev = self._host_t = None     # a whole-step graph capture / plan recording: no timing events
        elif self.cuda:
            self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            self._ev[0].record()
        else:
            self._host_t = [time.perf_counter(), None, None]
        if self.p2p is not None:
            self.p2p.begin_step()
        if self.mode == "sync":
            self.ex.grad_ready = self._on_ready
        else:
            self.ex.grad_ready = None

    def _launch(self, i: int, buf: Optional[torch.Tensor] = None, final: bool = False):
        lo, hi = self.buckets[i]
        if self.p2p is not None:
            side = self.ex.side
            self.p2p.reduce_bucket(i, lo, hi, after=(side,) if side is not None else (), final=final)
            self.launched[i] = True
            return
        t = (self.P.grad if buf is None else buf)[lo:hi]
        if self.wire_buf is not None and buf is None:
            w = self.wire_buf[lo:hi]
            self.ex.be.cast_bf16(t, w)         # fp32 -> bf16 (RNE), in-tree kernel, stream-ordered
            self.works.append(dist.all_reduce(w, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self.launched[i] = True
            return
        if self._sharded(lo, hi):
            # in place: this rank's shard of the bucket receives the sum over ranks
            s0, s1 = self._shard(lo, hi)
            out = (self.P.grad if buf is None else buf)[s0:s1]
            self.works.append(dist.reduce_scatter_tensor(out, t, op=dist.ReduceOp.SUM, group=self.group,
                                                         async_op=True))
        else:
            self.works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.launched[i] = True

    def _on_ready(self, lo_ready: int):
        self.frontier = min(self.frontier, lo_ready)
        for i, (lo, hi) in enumerate(self.buckets):
            if not self.launched[i] and lo >= self.frontier:
                self._launch(i)

    @property
    def wants_report_stream(self) -> bool:
        """Whether the executor issues this engine's bucket launches from its report stream
        (host-issued collectives); the P2P all-reduce orders its comm stream after the compute
        streams itself (P2PAllReduce.reduce_bucket)."""
        return self.p2p is None

    def launches_at(self, lo_ready: int) -> bool:
        """Whether a grad_ready(lo_ready) report would launch a bucket (the executor orders the
        report after the main stream only then: a report that launches nothing needs no
        cross-stream wait)."""
        f = min(self.frontier, lo_ready)
        return any(not self.launched[i] and lo >= f for i, (lo, _) in enumerate(self.buckets))

    def _mark(self, k: int):
        if self._ev is not None:
            self._ev[k].record()
        elif self._host_t is not None:
            self._host_t[k] = time.perf_counter()

    def _done(self):
        self._mark(2)
        if self.watchdog is not None:
            self.watchdog.done(self._ev[2] if self._ev is not None else None)

    def finish(self) -> torch.Tensor:
        """Complete the step's gradient exchange; returns the gradient buffer SGD must use."""
        if self.mode == "sync":
            for i in range(len(self.buckets)):
                if not self.launched[i]:
                    self._launch(i, final=True)
            self._mark(1)                      # backward done (all buckets issued)
            for w in self.works:
                w.wait()
            self._done_works, self.works = self.works, []
            self.ex.grad_ready = None
            if self.p2p is not None:
                self.p2p.end_step()
                self._done()
                return self.p2p.out
            self._done()
            return self.wire_buf if self.wire_buf is not None else self.P.grad
        # delayed (async-PS analog): finish last step's exchange, start this step's
        self._mark(1)
        for w in self.works:
            w.wait()
        self._done_works, self.works = self.works, []
        self._done()
        had = self._delayed_pending
        if had:
            self.ready_grad.copy_(self.comm_grad)
        else:
            self.ready_grad.zero_()
        self.comm_grad.copy_(self.P.grad)
        for i in range(len(self.buckets)):
            self._launch(i, self.comm_grad)
        self._delayed_pending = True
        return self.ready_grad

    def apply_gradients(self, grad: torch.Tensor, grad_scale: float):
        """The optimizer step after finish(): the executor's fused update (plain data parallel), or
        -- ZeRO-1 -- the update of this rank's shards followed by the all-gather of the compute
        weights and the refresh of the data-gradient weights."""
        if not self.zero1:
            # P2P: the optimizer reads the exchange's error word and skips a failed step's update
            self.ex.apply_gradients(grad_scale=grad_scale, grad=grad,
                                    skip=self.p2p.err if self.p2p is not None else None)
            return
        for lo, hi in self.buckets:
            s0, s1 = self._shard(lo, hi)
            self.ex.sgd_range(s0, s1, grad_scale, grad=grad)
        src = self.P.wbf16 if self.P.wbf16 is not None else self.P.master
        works = []
        for lo, hi in self.buckets:
            if self._sharded(lo, hi):
                s0, s1 = self._shard(lo, hi)
                works.append(dist.all_gather_into_tensor(src[lo:hi], src[s0:s1], group=self.group, async_op=True))
        for w in works:
            w.wait()
        self.ex.refresh_dgrad_weights()

    def gather_state(self):
        """ZeRO-1: make the fp32 masters and momentum complete on every rank (collective; before a
        checkpoint or anything else that reads them). No-op otherwise."""
        if not self.zero1:
            return
        for t in (self.P.master, self.P.momentum):
            for lo, hi in self.buckets:
                if self._sharded(lo, hi):
                    s0, s1 = self._shard(lo, hi)
                    dist.all_gather_into_tensor(t[lo:hi], t[s0:s1], group=self.group)

    def agree(self, flag: bool) -> bool:
        """Rank 0's decision, on every rank (collective)."""
        dev = self.P.master.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0, group=self.group)
        return bool(t.item())

    # -- whole-step graph replays (P2P data parallelism) ---------------------------------------------
    def replay_begin(self):
        """Host bookkeeping that the captured step no longer runs: the step counter and the
        collective watchdog's arm (a replayed step re-arms it like an eager one)."""
        self._step_no += 1
        if self.watchdog is not None:
            self.watchdog.arm(self._step_no)

    def replay_end(self):
        if self.watchdog is not None:
            ev = torch.cuda.Event() if self.cuda else None
            if ev is not None:
                ev.record()
            self.watchdog.done(ev)

    def poll_errors(self):
        """Non-blocking check of the P2P error word of completed steps (raises on failure)."""
        if self.p2p is not None:
            self.p2p.poll()

    def check_errors(self):
        """Synchronous check (before a checkpoint is written)."""
        if self.p2p is not None:
            self.p2p.check()

    def stats(self) -> dict:
        """Timing of the last completed step (synchronizes on its events)."""
        out = {"allreduce_buckets": len(self.buckets)}
        if self._ev is not None:
            self._ev[2].synchronize()
            bwd = self._ev[0].elapsed_time(self._ev[1])
            exposed = self._ev[1].elapsed_time(self._ev[2])
        elif self._host_t is not None and self._host_t[2] is not None:
            bwd = (self._host_t[1] - self._host_t[0]) * 1e3
            exposed = (self._host_t[2] - self._host_t[1]) * 1e3
        else:
            return out
        out["backward_ms"] = bwd
        out["comm_exposed_ms"] = max(exposed, 0.0)
        works = getattr(self, "_done_works", [])
        d = [_work_ms(w) for w in works]
        if d and all(x is not None for x in d):
            total = float(sum(d))      # RCCL kernel time (TORCH_NCCL_ENABLE_TIMING=1)
            out["comm_ms"] = total
            out["overlap_fraction"] = max(0.0, 1.0 - out["comm_exposed_ms"] / total) if total > 0 else 1.0
        return out

    def close(self):
        if self.watchdog is not None:
            self.watchdog.close()
            self.watchdog = None
        if self.p2p is not None:
            self.p2p.close()

    # -- state sync -----------------------------------------------------------------------------------
    def broadcast_parameters(self, src: int = 0):
        """Rank-0 broadcast of every variable (Horovod BroadcastGlobalVariablesHook(0) analog)."""
        for t in (self.P.master, self.P.momentum, self.P.bn_state):
            dist.broadcast(t, src=src, group=self.group)
        step = torch.tensor([self.P.global_step], dtype=torch.int64,
                            device=self.P.master.device)
        dist.broadcast(step, src=src, group=self.group)
        self.P.global_step = int(step.item())
        self.ex.sync_weights()

    def average_bn_state(self):
        """Optional: average BN moving statistics before checkpoint/eval (the reference keeps them
        per replica and checkpoints the chief's copy, so this is off by default)."""
        dist.all_reduce(self.P.bn_state, op=dist.ReduceOp.SUM, group=self.group)
        self.P.bn_state.div_(self.world)


def _work_ms(w) -> Optional[float]:
    """Device time of a finished collective when the process group records it (RCCL with
    TORCH_NCCL_ENABLE_TIMING=1); None otherwise."""
    try:
        d = w._get_duration()
        return float(d) if d is not None and d >= 0 else None
    except Exception:
        return None
