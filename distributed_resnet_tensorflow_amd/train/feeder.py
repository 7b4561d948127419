"""Moves host batches into the executor's fixed input buffers.

GPU path: host batch -> pinned staging tensors -> async H2D copy on a side stream (overlaps the
previous step's compute) -> GPU preprocessing kernel (CIFAR crop/flip/standardize, or the
fused VGG resize/crop/flip/mean-sub) writing NHWC bf16 (C padded to 8) straight into
`executor.images`. CPU path: the reference backend runs the same preprocessing in fp32.
Synthetic mode fills the device batch once (benchmarks: BASELINE "synthetic data").
"""
from __future__ import annotations

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

    def state(self):
        return {}

    def close(self):
        pass


class CifarFeeder:
    def __init__(self, ex, loader: "cifar_data.CifarLoader", is_training: bool):
        self.ex, self.loader, self.train = ex, loader, is_training
        N = ex.N
        dev = ex.device
        self.gpu = dev.type == "cuda"
        pin = self.gpu
        self.h_img = torch.empty(N, 32, 32, 3, dtype=torch.uint8, pin_memory=pin)
        self.h_lab = torch.empty(N, dtype=torch.int32, pin_memory=pin)
        self.h_par = torch.empty(N, 3, dtype=torch.int32, pin_memory=pin)
        self.d_img = torch.empty(N, 32, 32, 3, dtype=torch.uint8, device=dev)
        self.d_par = torch.empty(N, 3, dtype=torch.int32, device=dev)
        self.d_lab = torch.empty(N, dtype=torch.int32, device=dev)
        self.copy_stream = torch.cuda.Stream(device=dev) if self.gpu else None
        self._pending = None
        self._prefetch()

    def _prefetch(self):
        imgs, labels, params = next(self.loader)
        if self.gpu:
            # the previous batch's consumers (augment kernel) must be done with the staging tensors
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.ex.device))
            self.h_img.numpy()[...] = imgs
            self.h_lab.numpy()[...] = labels
            self.h_par.numpy()[...] = params
            with torch.cuda.stream(self.copy_stream):
                self.d_img.copy_(self.h_img, non_blocking=True)
                self.d_par.copy_(self.h_par, non_blocking=True)
                self.d_lab.copy_(self.h_lab, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self._pending = ev
        else:
            self.d_img.copy_(torch.from_numpy(imgs))
            self.d_par.copy_(torch.from_numpy(params))
            self.d_lab.copy_(torch.from_numpy(labels))

    def next(self):
        if self.gpu:
            torch.cuda.current_stream(self.ex.device).wait_event(self._pending)
        self.ex.be.cifar_augment(self.d_img, self.d_par, self.ex.images, cifar_data.PAD)
        self.ex.labels.copy_(self.d_lab)
        self._prefetch()
        return True

    def state(self):
        return self.loader.state()

    def close(self):
        self.loader.close()


class ImagenetFeeder:
    def __init__(self, ex, loader, is_training: bool, max_bytes: int = 64 << 20):
        from ..data import imagenet as inet
        self.inet = inet
        self.ex, self.loader = ex, loader
        self.gpu = ex.device.type == "cuda"
        self.d_buf = torch.empty(max_bytes, dtype=torch.uint8, device=ex.device)
        self.d_desc = torch.empty(ex.N * inet.IMG_DESC.itemsize, dtype=torch.uint8, device=ex.device)

    def next(self):
        try:
            packed, desc, labels = next(self.loader)
        except StopIteration:
            return False
        if self.gpu:
            if packed.size > self.d_buf.numel():
                self.d_buf = torch.empty(int(packed.size * 1.25), dtype=torch.uint8, device=self.ex.device)
            self.d_buf[:packed.size].copy_(torch.from_numpy(packed), non_blocking=False)
            self.d_desc.copy_(torch.from_numpy(desc.view(np.uint8)))
            self.ex.be.vgg_preprocess(self.d_buf, self.d_desc, self.ex.images, self.inet.RGB_MEANS)
        else:
            self.ex.be.vgg_preprocess(packed, desc, self.ex.images, self.inet.RGB_MEANS)
        self.ex.labels.copy_(torch.from_numpy(labels))
        return True

    def state(self):
        return {}

    def close(self):
        self.loader.close()
