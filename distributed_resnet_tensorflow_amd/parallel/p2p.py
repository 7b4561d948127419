"""One-shot peer-to-peer gradient all-reduce over xGMI (HIP IPC + csrc/kernels/allreduce_p2p.hip).

SURVEY §5.8 / §7.2 step 7: for small buckets (CIFAR ResNet's ~3 MB of fp32 gradients) a ring
all-reduce pays W-1 latency-bound steps per bucket; here each GPU maps every peer's gradient
buffer once (hipIpcGetMemHandle / hipIpcOpenMemHandle, handles exchanged over the existing
process group) and reduces a bucket in a single kernel that reads all peers concurrently. The
synchronisation is device-side (epoch flags in IPC-mapped memory), so the whole step, comm
included, stays capturable in one HIP graph. Buckets of at least `two_shot_min_kb`
(DRN_P2P_TWO_SHOT_MIN_KB, default 1024) use the two-shot form -- reduce-scatter of this rank's
1/W shard, then all-gather of the peers' reduced shards from their (also IPC-mapped) output
buffers -- which moves 2(W-1)/W of the bucket per GPU instead of (W-1)x.

Per step: ONE boundary kernel (publish DONE of the previous step, wait for every peer's DONE,
advance the device epoch) and ONE kernel per bucket (publish READY + wait + reduce; the two-shot
form adds the RS_DONE publish and the all-gather). `wire="bf16"` (DRN_P2P_WIRE=bf16) halves the
bytes every GPU pulls over xGMI: each bucket is first cast to a bf16 shadow buffer (also IPC-
mapped) on the compute stream and the peers read the shadows, accumulating in fp32 (the same
trade as Horovod's fp16 gradient compression).

Failure handling: every device-side wait is bounded in time (DRN_P2P_TIMEOUT_MS, default
60000). A timed-out wait sets the error word and returns; the optimizer launch reads the same
word and applies NO update (weights and momentum stay bitwise unchanged), and end_step() queues
a copy of the word into pinned host memory -- inside a captured HIP graph too -- which the
training session reads after every step without a device sync (poll()) and turns into an
exception; a checkpoint is only written after a synchronous check().

Memory: the flag arrays and the fp32 output buffers (read by the peers in the two-shot
all-gather) are UNCACHED device allocations (drn_p2p_alloc), exported by IPC: peer stores over
xGMI and local polling loads meet in memory, with no stale XCD-L2 copy on either side.

Limits: one node, <= 8 ranks, fp32 buckets whose element count is a multiple of 4.
"""
from __future__ import annotations

import ctypes
import logging
import os
import pickle

import torch
import torch.distributed as dist

from ..ops import _lib

log = logging.getLogger("drn")

MAX_RANKS = 8
N_SLOTS = 64          # ready slots (one per bucket) + the DONE slot 0
N_KINDS = 3           # READY, DONE, RS_DONE (two-shot)
_HIP = None


class _IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_uint8 * 64)]  # c_uint8, not c_char: handles contain NUL bytes

    @classmethod
    def from_bytes(cls, b: bytes) -> "_IpcHandle":
        h = cls()
        ctypes.memmove(ctypes.addressof(h), b, 64)
        return h

    def to_bytes(self) -> bytes:
        return ctypes.string_at(ctypes.addressof(self), 64)


class P2PArgs(ctypes.Structure):
    _fields_ = [
        ("out", ctypes.c_void_p),
        ("inp", ctypes.c_void_p * MAX_RANKS),
        ("out_peer", ctypes.c_void_p * MAX_RANKS),
        ("flags_local", ctypes.c_void_p),
        ("flags_peer", ctypes.c_void_p * MAX_RANKS),
        ("epoch", ctypes.c_void_p),
        ("err", ctypes.c_void_p),
        ("n", ctypes.c_int64),
        ("world", ctypes.c_int), ("rank", ctypes.c_int), ("slot", ctypes.c_int), ("timeout_ms", ctypes.c_int),
    ]


def _hip():
    global _HIP
    if _HIP is None:
        h = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_IpcHandle), ctypes.c_void_p]
        h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), _IpcHandle, ctypes.c_uint]
        h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
        h.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.c_void_p]
        for f in ("hipIpcGetMemHandle", "hipIpcOpenMemHandle", "hipIpcCloseMemHandle", "hipMemGetAddressRange"):
            getattr(h, f).restype = ctypes.c_int
        _HIP = h
    return _HIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def _export(t: torch.Tensor):
    """(ipc handle bytes, byte offset of t inside its allocation)."""
    h = _hip()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    _check(h.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(t.data_ptr())),
           "hipMemGetAddressRange")
    handle = _IpcHandle()
    _check(h.hipIpcGetMemHandle(ctypes.byref(handle), base), "hipIpcGetMemHandle")
    return handle.to_bytes(), t.data_ptr() - base.value


class _DeviceBuffer:
    """An uncached device allocation exposed to torch through __cuda_array_interface__ (the
    tensor does not own it: keep this object alive, release() frees it)."""

    def __init__(self, L, numel: int, dtype: torch.dtype, device: torch.device):
        self.L = L
        esize = torch.empty((), dtype=dtype).element_size()
        p = ctypes.c_void_p()
        _lib.check(L.drn_p2p_alloc(ctypes.byref(p), max(1, numel) * esize), "drn_p2p_alloc (uncached)")
        self.ptr = p.value
        typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]
        self.__cuda_array_interface__ = {"shape": (numel,), "typestr": typestr, "data": (self.ptr, False),
                                         "version": 2, "strides": None}
        self.tensor = torch.as_tensor(self, device=device)
        if self.tensor.data_ptr() != self.ptr or self.tensor.device.type != "cuda":
            raise RuntimeError("uncached P2P buffer could not be wrapped as a device tensor")

    def release(self):
        if self.ptr is not None:
            self.tensor = None
            self.L.drn_p2p_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


class P2PAllReduce:
    """Maps every rank's `grad` (and flag words) and reduces buckets of it into `out`."""

    _count = 0
    INLINE_MAX_MB = 16

    def __init__(self, grad: torch.Tensor, group=None, two_shot_min_kb: int = -1, wire: str = ""):
        P2PAllReduce._count += 1
        self._inst = P2PAllReduce._count
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > MAX_RANKS:
            raise ValueError("the P2P all-reduce supports one node of <= 8 ranks")
        self.L = _lib.lib()
        if self.L.drn_p2p_args_size() != ctypes.sizeof(P2PArgs):
            raise RuntimeError("P2PArgs layout mismatch between Python and the kernel library")
        self.grad = grad
        self._arg_cache = {}
        self.comm = torch.cuda.Stream(device=grad.device)
        # Where the bucket reductions run. On the P2P comm stream they overlap the rest of the
        # backward pass, but every bucket then costs two cross-queue hand-offs (compute -> comm ->
        # compute): CIFAR ResNet-50 bs32 at world 1, 1.85-1.94 ms per step vs 1.61 ms with the
        # reductions on the compute stream itself, i.e. the single-GPU rate 1.59 ms
        # (profiles/r6_p2p_plan_queues.txt). A small gradient's buckets reduce in microseconds and
        # the peers reach them together, so "auto" runs them inline up to INLINE_MAX_MB of
        # gradient; larger ones keep the comm stream (DRN_P2P_INLINE=auto | 1 | 0).
        mode = os.environ.get("DRN_P2P_INLINE", "auto").lower()
        self.inline = (mode == "1") or (mode == "auto" and grad.numel() * 4 <= self.INLINE_MAX_MB * (1 << 20))
        # cross-stream ordering: torch's stream API, or a native plan's recorder while a StepPlan
        # records the step (runtime/plan.py: the bucket kernels are then replayed from C++ too)
        self.sched = None
        dev = grad.device
        self.two_shot_min = 1024 * (two_shot_min_kb if two_shot_min_kb >= 0 else
                                    int(os.environ.get("DRN_P2P_TWO_SHOT_MIN_KB", "1024")))
        self.wire = (wire or "fp32").lower()
        if self.wire not in ("fp32", "bf16"):
            raise ValueError(f"P2P wire type must be fp32 or bf16, got {self.wire!r}")
        self.timeout_ms = int(os.environ.get("DRN_P2P_TIMEOUT_MS", "60000"))
        # fault injection (tests): "rank:bucket" -- that rank never launches that bucket's reduce,
        # i.e. never publishes it (eager steps only; a stuck peer as the other ranks see it)
        wh = os.environ.get("DRN_FAULT_P2P_WITHHOLD", "")
        self.withhold = int(wh.split(":")[1]) if wh and int(wh.split(":")[0]) == self.rank else -1
        self._bufs = [_DeviceBuffer(self.L, grad.numel(), torch.float32, dev),
                      _DeviceBuffer(self.L, N_SLOTS * N_KINDS * MAX_RANKS, torch.int32, dev)]
        self.out = self._bufs[0].tensor
        self.flags = self._bufs[1].tensor
        self.epoch = torch.zeros(1, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        # pinned host copy of the error word, refreshed by every step's end_step() (graph too)
        self.err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        # the tensor the peers read: the fp32 gradient itself, or its bf16 wire shadow
        self.shadow = torch.zeros(grad.numel(), dtype=torch.bfloat16, device=dev) if self.wire == "bf16" else None
        src = self.shadow if self.shadow is not None else grad
        self.esize = src.element_size()
        mine = (_export(src), _export(self.flags), _export(self.out))
        allh = [None] * self.world
        dist.all_gather_object(allh, pickle.dumps(mine), group=group)
        self._opened = []
        self.in_ptr, self.flag_ptr, self.out_ptr = [], [], []
        h = _hip()
        for r, blob in enumerate(allh):
            (gh, goff), (fh, foff), (oh, ooff) = pickle.loads(blob)
            if r == self.rank:
                self.in_ptr.append(src.data_ptr())
                self.flag_ptr.append(self.flags.data_ptr())
                self.out_ptr.append(self.out.data_ptr())
                continue
            ptrs, bases = [], {}   # buffers may share one allocation: open each handle once
            for hb, off in ((gh, goff), (fh, foff), (oh, ooff)):
                if hb not in bases:
                    hd = _IpcHandle.from_bytes(hb)
                    p = ctypes.c_void_p()
                    _check(h.hipIpcOpenMemHandle(ctypes.byref(p), hd, 1), "hipIpcOpenMemHandle")  # lazy peer access
                    self._opened.append(p.value)
                    bases[hb] = p.value
                ptrs.append(bases[hb] + off)
            self.in_ptr.append(ptrs[0])
            self.flag_ptr.append(ptrs[1])
            self.out_ptr.append(ptrs[2])
        dist.barrier(group=group)

    def _args(self, lo: int, hi: int, slot: int) -> P2PArgs:
        """Kernel argument block of (lo, hi, slot), built once and cached (the host launch path is
        on every eager step's critical path)."""
        key = (lo, hi, slot)
        a = self._arg_cache.get(key)
        if a is None:
            a = self._arg_cache[key] = self._make_args(lo, hi, slot)
        return a

    def _make_args(self, lo: int, hi: int, slot: int) -> P2PArgs:
        a = P2PArgs()
        a.out = self.out.data_ptr() + lo * 4
        for r in range(self.world):
            a.inp[r] = self.in_ptr[r] + lo * self.esize
            a.out_peer[r] = self.out_ptr[r] + lo * 4
            a.flags_peer[r] = self.flag_ptr[r]
        a.flags_local = self.flags.data_ptr()
        a.epoch = self.epoch.data_ptr()
        a.err = self.err.data_ptr()
        a.n = hi - lo
        a.world, a.rank, a.slot = self.world, self.rank, slot
        a.timeout_ms = self.timeout_ms
        return a

    @staticmethod
    def _stream():
        return torch.cuda.current_stream().cuda_stream

    def begin_step(self):
        """Before this step writes the gradient buffer: publish DONE for the previous step and
        wait until every peer finished reading this rank's buffers (one launch)."""
        a = self._args(0, 4, 0)
        _lib.check(self.L.drn_p2p_step(ctypes.byref(a), ctypes.c_void_p(self.epoch.data_ptr()), self._stream()),
                   "drn_p2p_step")

    def reduce_bucket(self, i: int, lo: int, hi: int, after=(), final: bool = False):
        """Bucket i = grad[lo:hi] is complete on the current stream and on the `after` streams
        (the executor's weight-gradient side stream): the comm stream waits for all of them, then
        (bf16 wire: casts the bucket to the shadow and) ONE kernel publishes it, polls for the
        peers without blocking the rest of this rank's backward pass, and reduces. No separate
        report stream: every stream a step uses is one more hardware queue, and with short CIFAR
        kernels each extra queue's cross-stream waits cost (profiles/r6_p2p_plan_queues.txt).
        final: a bucket launched after the backward pass (engine.finish) runs on the current
        stream itself -- nothing is left to overlap with, and the optimizer right behind it is
        then not two cross-queue hand-offs (there and back) away from its input."""
        assert (hi - lo) % 4 == 0 and lo % 4 == 0 and i + 1 < N_SLOTS
        if i == self.withhold:
            return  # fault injection: this rank never publishes bucket i
        a = self._args(lo, hi, i + 1)
        cur = torch.cuda.current_stream()
        st = cur if (final or self.inline) else self.comm
        if st is not cur:
            self._wait_stream(st, cur)
        for s in after:
            self._wait_stream(st, s)
        bf16 = self.shadow is not None
        if bf16:
            _lib.check(self.L.drn_p2p_cast(ctypes.c_void_p(self.grad.data_ptr() + lo * 4),
                                           ctypes.c_void_p(self.shadow.data_ptr() + lo * 2), hi - lo,
                                           st.cuda_stream), "drn_p2p_cast")
        # at most 128 workgroups: a reduce waiting for a slow peer must leave most CUs to this
        # rank's own backward kernels (which publish the later buckets the peers wait for)
        blocks = max(1, min(128, (hi - lo) // 4 // 256))
        if (hi - lo) * 4 >= self.two_shot_min and self.world > 1:
            _lib.check(self.L.drn_p2p_reduce2(ctypes.byref(a), blocks, int(bf16), st.cuda_stream),
                       "drn_p2p_reduce2")
        else:
            _lib.check(self.L.drn_p2p_reduce(ctypes.byref(a), blocks, int(bf16), st.cuda_stream),
                       "drn_p2p_reduce")

    def end_step(self):
        """All buckets reduced on this rank: order the compute stream after the reductions (the
        DONE publish happens at the next step's boundary launch) and queue the copy of the error
        word into pinned host memory (read by poll() without a device sync)."""
        cur = torch.cuda.current_stream()
        if not self.inline:
            self._wait_stream(cur, self.comm)
        if self.sched is None:          # (a replayed plan queues the copy itself: StepPlan.replay)
            self.err_host.copy_(self.err, non_blocking=True)

    def _wait_stream(self, dst, src):
        if self.sched is None:
            dst.wait_stream(src)
        else:
            self.sched.wait_stream(dst, src)

    @staticmethod
    def _raise(e: int):
        what = {1: "a bucket's READY", 2: "the step boundary's DONE", 3: "a two-shot RS_DONE"}.get(e, "a peer")
        raise RuntimeError(f"P2P all-reduce timed out waiting for {what} (code {e}): a peer rank is gone or "
                           f"stuck; the step's update was not applied")

    def poll(self):
        """Non-blocking: raise if the error word of an already completed step is set (at most a
        step or two behind the host; the update of any failed step was skipped on the device)."""
        e = int(self.err_host[0])
        if e:
            self._raise(e)

    def check(self):
        """Synchronous: raise if any device-side wait so far timed out (before a checkpoint)."""
        e = int(self.err.item())
        if e:
            self._raise(e)

    def close(self):
        """Collective teardown: unmap the peers' buffers, wait until every rank has done the
        same (nobody maps this rank's exported memory any more), then free it."""
        if torch.cuda.is_available():
            torch.cuda.synchronize(self.grad.device)
        h = _hip()
        for p in self._opened:
            h.hipIpcCloseMemHandle(ctypes.c_void_p(p))
        self._opened = []
        if self.world > 1:
            # time-bounded: a peer that failed (and skipped its close) must not hold this rank in
            # a collective until the process-group timeout; without the barrier the exported
            # buffers are left to process exit instead of being freed here
            try:
                self._store_barrier(60.0)
            except Exception as e:  # noqa: BLE001 -- any failure: keep the buffers mapped
                log.warning("P2P close: peers did not reach the teardown barrier (%s); buffers left to exit", e)
                self._leaked, self._bufs = self._bufs, []   # (no release: a peer may still map them)
                return
        for b in self._bufs:
            b.release()
        self._bufs = []

    def _store_barrier(self, timeout_s: float):
        """A barrier over the process group's TCPStore with a deadline (no collective kernel, so it
        also works after a device-side failure). Every rank adds 1 to a per-close key and polls."""
        import time
        store = dist.distributed_c10d._get_default_store()
        # (the same key on every rank: instances are created in the same order on all of them)
        key = f"drn_p2p_close/{self._inst}"
        store.add(key, 1)
        deadline = time.monotonic() + timeout_s
        while int(store.add(key, 0)) < self.world:
            if time.monotonic() > deadline:
                raise TimeoutError(f"{key}: {int(store.add(key, 0))}/{self.world} ranks after {timeout_s:.0f} s")
            time.sleep(0.01)
