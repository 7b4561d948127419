"""Moves host batches into the executor's fixed input buffers.

GPU path: host batch -> pinned staging tensors -> async H2D copy on a side stream (overlaps the
previous step's compute) -> GPU preprocessing kernel (CIFAR crop/flip/standardize, or the
fused VGG resize/crop/flip/mean-sub) writing NHWC bf16 (C padded to 8) straight into
`executor.images`. CPU path: the reference backend runs the same preprocessing in fp32.
Synthetic mode fills the device batch once (benchmarks: BASELINE "synthetic data").
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..data import cifar as cifar_data


class SyntheticFeeder:
    def __init__(self, ex, seed: int = 0):
        self.ex = ex
        ex.be.synthetic_images(ex.images, seed)
        g = torch.Generator().manual_seed(seed)
        ex.labels.copy_(torch.randint(0, ex.spec.num_classes, (ex.N,), generator=g, dtype=torch.int32))

    def next(self):
        return True

    def prefetch(self):
        pass

    def state(self):
        return {}

    def close(self):
        pass


def _as_tensor(x):
    return x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))


class _StagedFeeder:
    """Common GPU staging: batch k+1 is copied host->device on a side stream while step k runs.

    The loaders hand out a fresh page-locked buffer per batch (PyTorch's caching host
    allocator keeps a block out of circulation until the async copies recorded on it complete),
    so host-side writes can never race an in-flight DMA however far the host runs ahead of the
    GPU (graph replay). The device-side staging buffers are reused: a copy into them waits for
    the main stream's consumers of the previous batch (copy_stream.wait_stream).

    `state()` is the loader position after the batch most recently handed to the executor (not
    after the batch being prefetched), so a checkpoint resumes with the next unconsumed batch;
    `valid` is that batch's number of real (non-wrapped) images.

    Ordering (reference resnet_cifar_main.py:229-232 overlaps input with compute by
    `prefetch(2*batch_size)`): `next()` only hands batch k to the executor (stream-ordered
    preprocess kernel); the host-side load of batch k+1 runs in `prefetch()`, which the training
    session calls AFTER it has enqueued step k, so the host reads and decodes while the GPU
    computes. The H2D copies of batch k+1 wait only for the preprocess of batch k (an event), not
    for the whole step. A caller that never calls `prefetch()` gets it at the next `next()`.

    COPY_STREAM: whether the H2D copies get a stream of their own. Off for CIFAR (a batch is
    ~100 KB, a few microseconds of copy): the copies go on the consuming stream instead. A fifth
    busy stream in the process (beside the critical-path, weight-gradient, report and RCCL
    streams) shares one of the GPU_MAX_HW_QUEUES=4 hardware queues with a compute stream, and the
    cross-stream waits then serialise them: the CIFAR ResNet-50 bs32 CLI over RCCL ran 9.15 ms per
    step with the copy stream vs 2.05 ms without it, single-GPU 1.92 vs 1.81 ms
    (profiles/r5_cli_step_rate.txt). On for ImageNet, whose tens of MB per batch must overlap,
    as a HIGH-priority stream (COPY_STREAM_PRIORITY, DRN_COPY_STREAM_PRIORITY): that pool holds
    only the critical-path stream, so the copy stream shares no queue with a normal-priority
    compute stream. The ImageNet data-parallel step with the feeder: 10.09-10.10 ms vs 11.6 ms
    with a normal-priority copy stream (15.0-15.5 ms as a native plan) and 9.93 ms without
    copies (scripts/imagenet_copy_stream_probe.py, profiles/r6_imagenet_copy_stream.jsonl).
    """
    COPY_STREAM = True
    COPY_STREAM_PRIORITY = -1

    def _init_staging(self, ex):
        self.ex = ex
        self.gpu = ex.device.type == "cuda"
        prio = int(os.environ.get("DRN_COPY_STREAM_PRIORITY", str(self.COPY_STREAM_PRIORITY)))
        self.copy_stream = (torch.cuda.Stream(device=ex.device, priority=prio)
                            if self.gpu and self.COPY_STREAM else None)
        self._pending = None
        self._consumed = None          # event after the preprocess of the batch last handed out
        self._main = None              # the stream that consumes the batches (set by next())
        self._need_prefetch = False
        self._pending_state, self._pending_valid = self.loader.state(), ex.N
        self._state, self.valid = self.loader.state(), ex.N
        self._exhausted = False

    def _stage(self, pairs):
        """pairs: [(device dst, host src)]; enqueues the copies on the copy stream (or, without
        one, on the consuming stream: stream order after the previous batch's preprocess and
        before the next one's; prefetch may run on a worker thread, hence the explicit stream)."""
        if self.gpu:
            if self.copy_stream is None:
                with torch.cuda.stream(self._main or torch.cuda.current_stream(self.ex.device)):
                    for dst, src in pairs:
                        dst.copy_(_as_tensor(src), non_blocking=True)
                self._pending = None
                return
            # the device staging buffers are free once the previous batch's preprocess has read them
            if self._consumed is not None:
                self.copy_stream.wait_event(self._consumed)
            else:
                self.copy_stream.wait_stream(torch.cuda.current_stream(self.ex.device))
            with torch.cuda.stream(self.copy_stream):
                for dst, src in pairs:
                    dst.copy_(_as_tensor(src), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self._pending = ev
        else:
            for dst, src in pairs:
                dst.copy_(_as_tensor(src))

    def _prefetch(self):
        try:
            item = next(self.loader)
        except StopIteration:
            self._exhausted = True
            return
        self._pending_state = self.loader.state()
        self._pending_valid = int(getattr(self.loader, "valid", self.ex.N))
        self._stage_item(item)

    def _wait(self):
        if self.gpu and self._pending is not None:
            torch.cuda.current_stream(self.ex.device).wait_event(self._pending)

    def next(self):
        if self._need_prefetch:
            self.prefetch()
        if self._exhausted:
            return False
        self._wait()
        self._consume()
        if self.gpu:
            self._main = torch.cuda.current_stream(self.ex.device)
            self._consumed = torch.cuda.Event()
            self._consumed.record(self._main)
        self._state, self.valid = self._pending_state, self._pending_valid
        self._need_prefetch = True
        return True

    def prefetch(self):
        """Host-side load + async H2D staging of the next batch (call after enqueueing the step
        that consumes the current one)."""
        if self._need_prefetch:
            self._need_prefetch = False
            self._prefetch()

    def state(self):
        return dict(self._state)

    def close(self):
        self.loader.close()


class CifarFeeder(_StagedFeeder):
    COPY_STREAM = False

    def __init__(self, ex, loader: "cifar_data.CifarLoader", is_training: bool):
        self.loader, self.train = loader, is_training
        N, dev = ex.N, ex.device
        self.d_img = torch.empty(N, 32, 32, 3, dtype=torch.uint8, device=dev)
        self.d_par = torch.empty(N, 3, dtype=torch.int32, device=dev)
        self.d_lab = torch.empty(N, dtype=torch.int32, device=dev)
        self._init_staging(ex)
        self._prefetch()

    def _stage_item(self, item):
        imgs, labels, params = item
        self._stage([(self.d_img, imgs), (self.d_par, params), (self.d_lab, labels)])

    def _consume(self):
        self.ex.be.cifar_augment(self.d_img, self.d_par, self.ex.images, cifar_data.PAD)
        self.ex.labels.copy_(self.d_lab)


class ImagenetFeeder(_StagedFeeder):
    def __init__(self, ex, loader, is_training: bool, max_bytes: int = 64 << 20):
        from ..data import imagenet as inet
        self.inet = inet
        self.loader = loader
        self.d_buf = torch.empty(max_bytes, dtype=torch.uint8, device=ex.device)
        self.d_desc = torch.empty(ex.N * inet.IMG_DESC.itemsize, dtype=torch.uint8, device=ex.device)
        self.d_lab = torch.empty(ex.N, dtype=torch.int32, device=ex.device)
        self.h_packed = None  # CPU path: the reference backend preprocesses from host memory
        self.h_desc = None
        self._init_staging(ex)
        self._prefetch()

    def _stage_item(self, item):
        packed, desc, labels = item
        n = int(packed.numel() if isinstance(packed, torch.Tensor) else packed.size)
        # a pinned loader hands desc as a raw-byte tensor, labels as an int32 tensor
        desc_bytes = desc if isinstance(desc, torch.Tensor) else desc.view(np.uint8)
        if not self.gpu:
            self.h_packed = packed
            self.h_desc = desc.numpy().view(self.inet.IMG_DESC) if isinstance(desc, torch.Tensor) else desc
            self.d_lab.copy_(_as_tensor(labels))
            return
        if n > self.d_buf.numel():
            # reallocation (prefetch may run on a worker thread, whose current stream is NOT the
            # consuming one): the old buffer is released only after the last preprocess that read
            # it -- the event next() recorded on the consuming stream -- and the new one is
            # marked in use by both streams that touch it, so the caching allocator never hands
            # its memory out early
            if self._consumed is not None:
                self._consumed.synchronize()
            else:
                torch.cuda.synchronize(self.ex.device)
            self.d_buf = torch.empty(int(n * 1.25), dtype=torch.uint8, device=self.ex.device)
            if self.copy_stream is not None:
                self.d_buf.record_stream(self.copy_stream)
            if self._main is not None:
                self.d_buf.record_stream(self._main)
        self._stage([(self.d_buf[:n], packed), (self.d_desc, desc_bytes), (self.d_lab, labels)])

    def _consume(self):
        if self.gpu:
            self.ex.be.vgg_preprocess(self.d_buf, self.d_desc, self.ex.images, self.inet.RGB_MEANS)
        else:
            self.ex.be.vgg_preprocess(self.h_packed, self.h_desc, self.ex.images, self.inet.RGB_MEANS)
        self.ex.labels.copy_(self.d_lab)
