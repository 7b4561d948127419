"""CIFAR-10/100 binary input pipeline.

Reference: `record_dataset`/`get_filenames`/`parse_record`/`preprocess_image`/`input_fn`
(resnet_cifar_main.py:134-246) and the queue-based `cifar_input.build_input` used by eval
(cifar_input.py:21-115).
  * files: <dir>/cifar-10-batches-bin/data_batch_{1..5}.bin (train), test_batch.bin (eval);
    a file glob (the eval scripts pass `--eval_data_path=.../test_batch*`) or a single file
    also works; CIFAR-100: train.bin / test.bin.
  * record: CIFAR-10 = 1 label byte + 3072 CHW bytes; CIFAR-100 = coarse + fine label bytes
    + 3072 (label_offset 1, cifar_input.py:40-49).
  * train: full-epoch shuffle (reference shuffle buffer = 50,000), pad 4 px/side, random
    32x32 crop, random left-right flip, per-image standardization (resnet_cifar_main.py:185-200;
    the +8 tf.data variant actually used for training); eval: standardization only.
Records are memory-mapped and gathered by the native host helper (CHW -> HWC) into pinned
uint8 batches; crop/flip/standardize run on the GPU (csrc/kernels/augment.hip) or, on the CPU
path, in the reference backend. Data-parallel ranks take disjoint shards of each epoch's
permutation (the reference's workers each shuffled the full set independently).
"""
from __future__ import annotations

import glob
import os
import threading
import queue
from typing import List, Optional, Tuple

import numpy as np

from ..utils.native import host_lib

HEIGHT = WIDTH = 32
DEPTH = 3
NUM_IMAGES = {"train": 50000, "validation": 10000}
PAD = 4


def record_layout(dataset: str) -> Tuple[int, int]:
    """(label_bytes, label_offset) of a record."""
    if dataset == "cifar100":
        return 2, 1
    return 1, 0


def get_filenames(is_training: bool, data_dir: str, dataset: str = "cifar10") -> List[str]:
    """reference get_filenames (resnet_cifar_main.py:140-154) + glob / file patterns."""
    if data_dir and (any(ch in data_dir for ch in "*?[") or os.path.isfile(data_dir)):
        files = sorted(glob.glob(data_dir))
        if files:
            return files
    if dataset == "cifar100":
        d = os.path.join(data_dir, "cifar-100-binary")
        d = d if os.path.isdir(d) else data_dir
        return [os.path.join(d, "train.bin" if is_training else "test.bin")]
    d = os.path.join(data_dir, "cifar-10-batches-bin")
    d = d if os.path.isdir(d) else data_dir
    if is_training:
        return [os.path.join(d, f"data_batch_{i}.bin") for i in range(1, 6)]
    return [os.path.join(d, "test_batch.bin")]


class CifarRecords:
    """All records of a set of CIFAR binary files, memory-mapped."""

    def __init__(self, files: List[str], dataset: str = "cifar10"):
        self.label_bytes, self.label_offset = record_layout(dataset)
        self.record_bytes = self.label_bytes + HEIGHT * WIDTH * DEPTH
        arrs = []
        for f in files:
            if not os.path.exists(f):
                raise FileNotFoundError(f)
            arrs.append(np.memmap(f, dtype=np.uint8, mode="r"))
        self.data = np.ascontiguousarray(np.concatenate(arrs)) if len(arrs) > 1 else np.asarray(arrs[0])
        if self.data.size % self.record_bytes:
            raise ValueError(f"file size is not a multiple of {self.record_bytes} bytes")
        self.n = self.data.size // self.record_bytes

    def gather(self, idx: np.ndarray, images: np.ndarray, labels: np.ndarray):
        """images [n,32,32,3] uint8 (HWC), labels [n] int32 for record indices idx."""
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        lib = host_lib()
        data = np.ascontiguousarray(self.data)
        if lib is not None:
            lib.drn_cifar_gather(data.ctypes.data, idx.ctypes.data, len(idx), self.record_bytes, self.label_bytes,
                                 self.label_offset, images.ctypes.data, labels.ctypes.data)
            return
        recs = data.reshape(self.n, self.record_bytes)[idx]
        labels[:] = recs[:, self.label_offset]
        images[:] = recs[:, self.label_bytes:].reshape(-1, DEPTH, HEIGHT, WIDTH).transpose(0, 2, 3, 1)


def _device_index(dev):
    """Integer GPU index of `dev` (None, 'cuda', 'cuda:1', torch.device, int); resolved on the
    constructing (main) thread so a loader thread can select the same device."""
    import torch
    if dev is None:
        return torch.cuda.current_device()
    if isinstance(dev, int):
        return dev
    d = torch.device(dev)
    return d.index if d.index is not None else torch.cuda.current_device()


def _host_array(shape, dtype, pin: bool):
    """(tensor-or-array, numpy view) of a fresh host buffer; page-locked when `pin`."""
    if not pin:
        a = np.empty(shape, dtype=dtype)
        return a, a
    import torch
    t = torch.empty(shape, dtype={np.uint8: torch.uint8, np.int32: torch.int32}[dtype], pin_memory=True)
    return t, t.numpy()


class CifarLoader:
    """Iterator of (uint8 HWC images, int32 labels, int32 aug params [n,3]) host batches.

    Train: epoch-wise shuffled, rank-sharded, drop-remainder; random crop offsets in [0, 2*PAD]
    and flip bits drawn from the seeded host RNG. Eval: sequential, no augmentation.
    A background thread keeps `prefetch` batches ready. With `pin=True` every batch is gathered
    straight into its own page-locked tensors (PyTorch's caching host allocator does not hand a
    block out again until the async copies recorded on it have completed, so a batch can never
    be overwritten while its DMA is in flight). Each batch carries the loader position *after*
    it (`state()` reports the position after the last batch handed out) and its number of
    valid (non-wrapped) images (`valid`: only the final partial eval batch has fewer).
    """

    def __init__(self, records: CifarRecords, batch_size: int, is_training: bool, seed: int = 0, rank: int = 0,
                 world: int = 1, prefetch: int = 4, epoch: int = 0, cursor: int = 0, pin: bool = False,
                 pin_device=None):
        self.rec = records
        self.pin, self.pin_device = pin, _device_index(pin_device) if pin else None
        self._error: Optional[BaseException] = None
        self.valid = batch_size
        self.bs = batch_size
        self.train = is_training
        self.seed, self.rank, self.world = seed, rank, world
        self.epoch, self.cursor = epoch, cursor
        self.q: "queue.Queue" = queue.Queue(maxsize=max(1, prefetch))
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _perm(self, epoch: int) -> np.ndarray:
        if not self.train:
            return np.arange(self.rec.n)
        rng = np.random.default_rng([self.seed, epoch])
        p = rng.permutation(self.rec.n)
        per = self.rec.n // self.world
        return p[self.rank * per:(self.rank + 1) * per]

    def _run(self):
        try:
            self._produce()
        except BaseException as e:  # surfaces in the consumer's next() instead of a silent hang
            self._error = e
            self.q.put(None)

    def _produce(self):
        if self.pin and self.pin_device is not None:
            import torch
            torch.cuda.set_device(self.pin_device)  # page-locked allocations in this rank's context
        epoch, cursor = self.epoch, self.cursor
        perm = self._perm(epoch)
        while not self._stop.is_set():
            valid = self.bs
            if cursor + self.bs > len(perm):
                if not self.train and cursor < len(perm):
                    idx = perm[cursor:]  # final partial eval batch, padded by wrapping around
                    valid = len(idx)
                    idx = np.concatenate([idx, perm[:self.bs - len(idx)]])
                else:
                    epoch += 1
                    cursor = 0
                    perm = self._perm(epoch)
                    continue
            else:
                idx = perm[cursor:cursor + self.bs]
            # crop/flip draws are a function of the batch position: a resumed loader is exact
            rng = np.random.default_rng([self.seed, 7919, self.rank, epoch, cursor])
            cursor += self.bs
            imgs, imgs_np = _host_array((self.bs, HEIGHT, WIDTH, DEPTH), np.uint8, self.pin)
            labels, labels_np = _host_array((self.bs,), np.int32, self.pin)
            self.rec.gather(idx, imgs_np, labels_np)
            if self.train:
                p = np.stack([rng.integers(0, 2 * PAD + 1, self.bs), rng.integers(0, 2 * PAD + 1, self.bs),
                              rng.integers(0, 2, self.bs)], axis=1).astype(np.int32)
            else:
                p = np.tile(np.array([[PAD, PAD, 0]], dtype=np.int32), (self.bs, 1))
            params, params_np = _host_array((self.bs, 3), np.int32, self.pin)
            params_np[...] = p
            item = (imgs, labels, params, epoch, cursor, valid)
            while not self._stop.is_set():
                try:
                    self.q.put(item, timeout=0.1)
                    break
                except queue.Full:
                    continue

    def __iter__(self):
        return self

    def __next__(self):
        item = self.q.get()
        if item is None:
            raise RuntimeError("CIFAR loader thread failed") from self._error
        imgs, labels, params, epoch, cursor, valid = item
        self.epoch, self.cursor, self.valid = epoch, cursor, valid
        return imgs, labels, params

    def state(self):
        return {"data_epoch": self.epoch, "data_cursor": self.cursor}

    def close(self):
        self._stop.set()
        self._t.join(timeout=2)


def write_fake_cifar(dirpath: str, n_per_file: int = 100, dataset: str = "cifar10", seed: int = 0,
                     learnable: bool = False) -> str:
    """Writes small CIFAR-format binary files (tests / smoke runs without the real dataset).
    `learnable`: every class has its own colour (per-channel offsets that survive the per-image
    standardisation, crops and flips) plus noise, so a trained model can reach high precision
    on the test file — a convergence check with no dataset available."""
    rng = np.random.default_rng(seed)
    lb, lo = record_layout(dataset)
    ncls = 100 if dataset == "cifar100" else 10
    if dataset == "cifar100":
        d = os.path.join(dirpath, "cifar-100-binary")
        names = ["train.bin", "test.bin"]
    else:
        d = os.path.join(dirpath, "cifar-10-batches-bin")
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]
    os.makedirs(d, exist_ok=True)
    for name in names:
        recs = np.zeros((n_per_file, lb + 3072), dtype=np.uint8)
        labels = rng.integers(0, ncls, n_per_file)
        recs[:, lo] = labels
        if lb == 2:
            recs[:, 0] = labels // 5
        if learnable:
            # hues evenly spaced around the colour wheel: distinct zero-mean channel patterns
            hue = 2 * np.pi * np.arange(ncls) / ncls
            palette = np.round(128 + 80 * np.cos(hue[:, None] - np.array([0, 2, 4]) * np.pi / 3)).astype(np.int64)
            base = np.repeat(palette[labels], 1024, axis=1)  # CHW: each channel plane its own value
            noise = rng.integers(-35, 36, (n_per_file, 3072))
        else:  # class-dependent mean so that a small model can learn something
            base = (labels[:, None] * 23) % 256
            noise = rng.integers(-40, 40, (n_per_file, 3072))
        recs[:, lb:] = np.clip(base + noise, 0, 255).astype(np.uint8)
        recs.tofile(os.path.join(d, name))
    return dirpath
