"""ImageNet TFRecord input pipeline + VGG preprocessing.

Reference: resnet_imagenet_main.py:103-183 (filenames / record_parser / input_fn) and
vgg_preprocessing.py:229-363.
  * shards <dir>/train-%05d-of-01024 and <dir>/validation-%05d-of-00128 (falls back to any
    `train-*` / `validation-*` files present);
  * tf.Example: 'image/encoded' (JPEG/PNG bytes), 'image/class/label' (int64, 1..1000 with
    0 = background -> 1001 classes); bounding boxes are parsed-and-ignored in the reference too;
  * train: file-order shuffle, example shuffle buffer 1500, smaller side resized to U{256..512}
    (aspect preserving, TF1 legacy bilinear), random 224 crop, random flip, RGB mean
    subtraction of (123.68, 116.78, 103.94)/255 on [0,1] pixels; eval: smaller side 256,
    central 224 crop, mean subtraction.
Host side: TFRecord scan (native CRC check), Example parsing, JPEG decode (PIL, thread pool)
and the per-image geometry draws. GPU side: one fused resize+crop+flip+mean-sub kernel over
the packed decoded batch (csrc/kernels/augment.hip, drn_vgg_preprocess); the CPU path runs the
same math in numpy (RefBackend.vgg_preprocess).
"""
from __future__ import annotations

import glob
import io
import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Tuple

import numpy as np

from ..utils import pbwire as pb
from ..utils.tfrecord import TFRecordWriter, read_records

IMAGE_SIZE = 224
NUM_CLASSES = 1001
NUM_IMAGES = {"train": 1281167, "validation": 50000}
FILE_SHUFFLE_BUFFER = 1024
SHUFFLE_BUFFER = 1500
RGB_MEANS = (123.68 / 255, 116.78 / 255, 103.94 / 255)
RESIZE_MIN, RESIZE_MAX = 256, 512

# numpy mirror of csrc/kernels/augment.hip `struct ImgDesc`
IMG_DESC = np.dtype([("offset", "<i8"), ("H", "<i4"), ("W", "<i4"), ("rh", "<i4"), ("rw", "<i4"),
                     ("cy", "<i4"), ("cx", "<i4"), ("flip", "<i4"), ("pad", "<i4")])


def filenames(is_training: bool, data_dir: str) -> List[str]:
    if is_training:
        names = [os.path.join(data_dir, "train-%05d-of-01024" % i) for i in range(1024)]
    else:
        names = [os.path.join(data_dir, "validation-%05d-of-00128" % i) for i in range(128)]
    if all(os.path.exists(n) for n in names):
        return names
    pat = "train-*" if is_training else "validation-*"
    found = sorted(glob.glob(os.path.join(data_dir, pat)))
    if found:
        return found
    raise FileNotFoundError(f"no ImageNet {'train' if is_training else 'validation'} shards in {data_dir}")


# -- tf.Example ------------------------------------------------------------------------------
# Example { Features features = 1 }  Features { map<string, Feature> feature = 1 }
# Feature { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3 }
def parse_example(buf: bytes) -> dict:
    out = {}
    ex = pb.decode(buf)
    for feats in ex.get(1, []):
        for entry in pb.decode(feats).get(1, []):
            e = pb.decode(entry)
            key = e[1][0].decode() if 1 in e else ""
            if 2 not in e:
                continue
            f = pb.decode(e[2][0])
            if 1 in f:
                out[key] = [bytes(v) for v in pb.decode(f[1][0]).get(1, [])]
            elif 3 in f:
                il = pb.decode(f[3][0]).get(1, [])
                vals = []
                for v in il:
                    if isinstance(v, (bytes, bytearray, memoryview)):  # packed
                        pos, b = 0, bytes(v)
                        while pos < len(b):
                            x, pos = pb.read_varint(b, pos)
                            vals.append(pb.signed64(x))
                    else:
                        vals.append(pb.signed64(v))
                out[key] = vals
            elif 2 in f:
                fl = pb.decode(f[2][0]).get(1, [])
                vals = []
                for v in fl:
                    b = bytes(v)
                    vals.extend(np.frombuffer(b, dtype="<f4").tolist())
                out[key] = vals
    return out


def make_example(image_bytes: bytes, label: int, fmt: str = "jpeg") -> bytes:
    def feat_bytes(b):
        return pb.f_bytes(1, pb.f_bytes(1, b))

    def feat_int(v):
        return pb.f_bytes(3, pb.f_bytes(1, pb.varint(v)))

    def entry(k, f):
        return pb.f_bytes(1, pb.f_string(1, k) + pb.f_bytes(2, f))

    feats = entry("image/encoded", feat_bytes(image_bytes)) + entry("image/format", feat_bytes(fmt.encode())) + \
        entry("image/class/label", feat_int(label))
    return pb.f_bytes(1, feats)


def decode_image(b: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(b)) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


# -- VGG geometry ------------------------------------------------------------------------------
def smallest_size_at_least(h: int, w: int, side: int) -> Tuple[int, int]:
    scale = side / w if h > w else side / h
    return int(h * scale), int(w * scale)


def draw_geometry(h: int, w: int, is_training: bool, rng: np.random.Generator, out: int = IMAGE_SIZE):
    side = int(rng.integers(RESIZE_MIN, RESIZE_MAX + 1)) if is_training else RESIZE_MIN
    rh, rw = smallest_size_at_least(h, w, side)
    if is_training:
        cy = int(rng.integers(0, rh - out + 1))
        cx = int(rng.integers(0, rw - out + 1))
        flip = int(rng.integers(0, 2))
    else:
        cy, cx, flip = (rh - out) // 2, (rw - out) // 2, 0
    return rh, rw, cy, cx, flip


def vgg_preprocess_np(img: np.ndarray, rh: int, rw: int, cy: int, cx: int, flip: int, out: int = IMAGE_SIZE):
    """CPU reference of the fused GPU kernel: legacy TF bilinear (src = dst*in/out), crop, flip,
    /255, mean subtraction. Returns float32 [out,out,3]."""
    H, W = img.shape[:2]
    ys = (np.arange(out) + cy) * (H / rh)
    xs_idx = np.arange(out)
    if flip:
        xs_idx = out - 1 - xs_idx
    xs = (xs_idx + cx) * (W / rw)
    y0 = np.clip(np.floor(ys).astype(np.int64), 0, H - 1)
    x0 = np.clip(np.floor(xs).astype(np.int64), 0, W - 1)
    y1 = np.minimum(y0 + 1, H - 1)
    x1 = np.minimum(x0 + 1, W - 1)
    wy = (ys - y0)[:, None, None].astype(np.float32)
    wx = (xs - x0)[None, :, None].astype(np.float32)
    f = img.astype(np.float32)
    a, b = f[y0][:, x0], f[y0][:, x1]
    c, d = f[y1][:, x0], f[y1][:, x1]
    top = a + (b - a) * wx
    bot = c + (d - c) * wx
    res = (top + (bot - top) * wy) / 255.0
    return res - np.array(RGB_MEANS, dtype=np.float32)


class _Shard:
    """Record index of one TFRecord shard: the file is memory-mapped and only the 12-byte
    record headers are walked (no payload read, no CRC) when the index is built; each record's
    CRCs are checked when it is fetched."""

    def __init__(self, path: str):
        self.path = path
        self._mm = None
        self.offsets: Optional[np.ndarray] = None  # frame offsets (header start)
        self.lengths: Optional[np.ndarray] = None

    def _map(self):
        if self._mm is None:
            import mmap
            with open(self.path, "rb") as f:
                size = os.fstat(f.fileno()).st_size
                self._mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
        return self._mm

    def count(self) -> int:
        if self.offsets is None:
            import struct
            mm = self._map()
            offs, lens, pos, n = [], [], 0, len(mm)
            while pos + 12 <= n:
                (ln,) = struct.unpack_from("<Q", mm, pos)
                if pos + 16 + ln > n:
                    raise IOError(f"truncated TFRecord {self.path} at byte {pos}")
                offs.append(pos)
                lens.append(ln)
                pos += 16 + ln
            self.offsets = np.asarray(offs, dtype=np.int64)
            self.lengths = np.asarray(lens, dtype=np.int64)
        return len(self.offsets)

    def record(self, i: int, check: bool = True) -> bytes:
        self.count()
        off, ln = int(self.offsets[i]), int(self.lengths[i])
        frame = self._map()[off:off + 16 + ln]
        if check:
            from ..utils.tfrecord import scan
            scan(frame, True)  # raises CorruptRecordError on a bad length / data CRC
        return frame[12:12 + ln]


_WORKER_SHARDS: dict = {}
_CHUNK = 8  # records per decode-process task
_SHM_PREFIX = "drn_dec_"
_SEQ = 0


def _decode_in_worker(path: str, r: int):
    """Decode-worker-process side of ImagenetLoader(workers="process"): read record r of the
    shard (its own memory map, CRC-checked), parse the Example, decode the JPEG. Module level
    and torch-free so a spawned worker imports only numpy / PIL / this package's codecs."""
    sh = _WORKER_SHARDS.get(path)
    if sh is None:
        sh = _WORKER_SHARDS[path] = _Shard(path)
    ex = parse_example(sh.record(r))
    img = decode_image(ex["image/encoded"][0])
    # the pixels travel through a shared-memory segment, not the result pipe: pickling ~0.5 MB
    # per image through the pool's single result thread capped the parent near 1k img/s. The
    # segment is named after the loader's process (cleanup of leftovers: _shm_cleanup) and is
    # owned by the parent, which unlinks it after copying: not tracked here.
    from multiprocessing import resource_tracker, shared_memory
    global _SEQ
    _SEQ += 1
    seg = shared_memory.SharedMemory(name=f"{_SHM_PREFIX}{os.getppid()}_{os.getpid()}_{_SEQ}", create=True,
                                     size=max(1, img.nbytes))
    resource_tracker.unregister(seg._name, "shared_memory")
    np.ndarray(img.shape, np.uint8, buffer=seg.buf)[...] = img
    name = seg.name
    seg.close()
    return (name, img.shape), int(ex.get("image/class/label", [-1])[0])


def _shm_cleanup(pid: int) -> None:
    """Unlink every decode segment created for loader process `pid` that is still in /dev/shm
    (batches decoded but never consumed when the loader stops)."""
    for f in glob.glob(f"/dev/shm/{_SHM_PREFIX}{pid}_*"):
        try:
            os.unlink(f)
        except OSError:
            pass


def _shm_cleanup_stale() -> int:
    """Unlink decode segments whose loader process no longer exists (a loader that died by
    SIGKILL, OOM or os._exit never ran its atexit cleanup). Segment names carry the loader's pid
    (`drn_dec_<loader pid>_<worker pid>_<seq>`). Returns the number of segments removed."""
    n = 0
    for f in glob.glob(f"/dev/shm/{_SHM_PREFIX}*"):
        try:
            pid = int(os.path.basename(f)[len(_SHM_PREFIX):].split("_", 1)[0])
        except ValueError:
            continue
        if pid == os.getpid():
            continue
        try:
            os.kill(pid, 0)
            continue                   # the loader is alive (this user's or another's): keep
        except ProcessLookupError:
            pass
        except PermissionError:
            continue                   # alive, owned by another user
        try:
            os.unlink(f)
            n += 1
        except OSError:
            pass
    return n


def _decode_chunk_in_worker(items):
    """Several records per task (fewer pool round trips): [(path, r)] -> [((shm, shape), label)]."""
    return [_decode_in_worker(p, r) for p, r in items]


class _ShmImage:
    """A decoded image left in a shared-memory segment by a decode worker: attached on the
    loader thread, copied into the batch buffer, then unlinked."""
    __slots__ = ("seg", "arr")

    def __init__(self, name: str, shape):
        from multiprocessing import shared_memory
        self.seg = shared_memory.SharedMemory(name=name)
        self.arr = np.ndarray(shape, np.uint8, buffer=self.seg.buf)

    def release(self):
        self.arr = None
        self.seg.close()
        self.seg.unlink()


class ImagenetLoader:
    """Background pipeline producing packed decoded batches:
    (packed uint8 buffer, IMG_DESC array [B], int32 labels [B]).

    The record order is a pure function of (seed, rank, epoch): per-epoch file shuffle, then the
    reference's 1500-deep example shuffle buffer (resnet_imagenet_main.py:165-173) run over
    (shard, record) *indices*. A position is therefore just (epoch, records consumed in the
    epoch), and resuming from a checkpoint skips that many indices without reading or decoding
    any image. Crop/flip geometry of batch b comes from an RNG seeded with (seed, rank, b). Each
    batch carries the position after it; `state()` reports the position after the last batch
    handed out. With `pin=True` batches are packed straight into page-locked tensors.

    workers="thread" decodes in a thread pool; "process" in spawned worker processes. JPEG
    decoding holds the GIL for part of each image (colour conversion, array copies): measured on
    8 cores (scripts/imagenet_input_bench.py, profiles/r3_imagenet_input_bench.txt) threads
    saturate near 1.3k img/s while processes scale ~linearly (~350 img/s per core for 500x375
    JPEGs), so training uses processes.
    """

    def __init__(self, data_dir: str, batch_size: int, is_training: bool, seed: int = 0, rank: int = 0,
                 world: int = 1, num_threads: int = 8, prefetch: int = 3, num_epochs: Optional[int] = None,
                 epoch: int = 0, cursor: int = 0, batch_index: int = 0, pin: bool = False, pin_device=None,
                 workers: str = "thread"):
        files = filenames(is_training, data_dir)
        if is_training and world > 1:
            files = files[rank::world] or files
        self.files = files
        self.shards = [_Shard(f) for f in files]
        self.bs, self.train, self.seed, self.rank = batch_size, is_training, seed, rank
        self.num_epochs = num_epochs
        from .cifar import _device_index
        self.pin, self.pin_device = pin, _device_index(pin_device) if pin else None
        self._error: Optional[BaseException] = None
        self.epoch, self.cursor, self.batch_index = epoch, cursor, batch_index
        if workers not in ("thread", "process"):
            raise ValueError(f"decode workers must be 'thread' or 'process', got {workers!r}")
        self.workers = workers
        if workers == "process":
            import atexit
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor
            # spawn: never fork a process that holds a GPU context
            self.pool = ProcessPoolExecutor(max_workers=max(1, num_threads), mp_context=mp.get_context("spawn"))
            atexit.register(_shm_cleanup, os.getpid())
            _shm_cleanup_stale()       # leftovers of loaders that died without their atexit
        else:
            self.pool = ThreadPoolExecutor(max_workers=max(1, num_threads))
        self.q: "queue.Queue" = queue.Queue(maxsize=max(1, prefetch))
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def epoch_order(self, epoch: int):
        """Yields the (shard, record) indices of one epoch in training order."""
        rng = np.random.default_rng([self.seed, self.rank, 17, epoch])
        order = list(range(len(self.shards)))
        if self.train:
            rng.shuffle(order)
        buf = []
        for s in order:
            for r in range(self.shards[s].count()):
                if not self.train:
                    yield s, r
                    continue
                buf.append((s, r))
                if len(buf) >= SHUFFLE_BUFFER:
                    j = int(rng.integers(0, len(buf)))
                    buf[j], buf[-1] = buf[-1], buf[j]
                    yield buf.pop()
        while buf:
            j = int(rng.integers(0, len(buf)))
            buf[j], buf[-1] = buf[-1], buf[j]
            yield buf.pop()

    def _positions(self):
        """(shard, record, epoch, cursor-after) from the resume position onwards."""
        epoch, skip = self.epoch, self.cursor
        while not self._stop.is_set():
            if self.num_epochs is not None and epoch >= self.num_epochs:
                return
            n = 0
            for s, r in self.epoch_order(epoch):
                n += 1
                if n <= skip:
                    continue
                yield s, r, epoch, n
            epoch, skip = epoch + 1, 0

    def _decode(self, pos):
        ex = parse_example(self.shards[pos[0]].record(pos[1]))
        img = decode_image(ex["image/encoded"][0])
        label = int(ex.get("image/class/label", [-1])[0])
        return img, label

    def _batches(self):
        """(futures of one batch's decodes, epoch, cursor-after), with the NEXT batch's decodes
        already submitted before the current one is handed on: the pool never idles on the
        slowest image of a batch (two batches in flight)."""
        inflight, batch = [], []
        for s, r, epoch, cursor in self._positions():
            batch.append((s, r))
            if len(batch) < self.bs:
                continue
            if self.workers == "process":
                items = [(self.shards[s].path, r) for s, r in batch]
                futs = [self.pool.submit(_decode_chunk_in_worker, items[i:i + _CHUNK])
                        for i in range(0, len(items), _CHUNK)]
            else:
                futs = [self.pool.submit(self._decode, pos) for pos in batch]
            inflight.append((futs, epoch, cursor))
            batch = []
            if len(inflight) > 1:
                yield inflight.pop(0)
        yield from inflight

    def _host(self, n: int, dtype):
        """A fresh host buffer (page-locked with pin=True, so its async H2D copy never stages
        through pageable memory): (object handed on, numpy view). Pinned int32 buffers are
        int32 tensors; other pinned dtypes are raw uint8 tensors."""
        if not self.pin:
            a = np.empty(n, dtype=dtype)
            return a, a
        import torch
        if np.dtype(dtype) == np.int32:
            t = torch.empty(n, dtype=torch.int32, pin_memory=True)
            return t, t.numpy()
        t = torch.empty(n * np.dtype(dtype).itemsize, dtype=torch.uint8, pin_memory=True)
        return t, t.numpy().view(dtype)

    def _run(self):
        b = self.batch_index
        try:
            if self.pin and self.pin_device is not None:
                import torch
                torch.cuda.set_device(self.pin_device)
            for futs, epoch, cursor in self._batches():
                shm = []
                if self.workers == "process":
                    decoded = [d for f in futs for d in f.result()]
                    shm = [_ShmImage(*ref) for ref, _ in decoded]
                    decoded = [(m.arr, lab) for m, (_, lab) in zip(shm, decoded)]
                else:
                    decoded = [f.result() for f in futs]
                rng = np.random.default_rng([self.seed, self.rank, 99, b])
                total = sum(d[0].size for d in decoded)
                packed, flat = self._host(total, np.uint8)
                desc_h, desc = self._host(self.bs, IMG_DESC)
                labels_h, labels = self._host(self.bs, np.int32)
                desc[...] = np.zeros((), dtype=IMG_DESC)
                off = 0
                for i, (img, lab) in enumerate(decoded):
                    h, w = img.shape[:2]
                    flat[off:off + img.size] = img.reshape(-1)
                    rh, rw, cy, cx, flip = draw_geometry(h, w, self.train, rng)
                    desc[i] = (off, h, w, rh, rw, cy, cx, flip, 0)
                    labels[i] = lab
                    off += img.size
                decoded = None
                for m in shm:
                    m.release()
                b += 1
                # pin=True: the page-locked tensors themselves (desc as raw IMG_DESC bytes), so the
                # caching host allocator tracks their async copies
                item = (packed, desc_h, labels_h, {"data_epoch": epoch, "data_cursor": cursor, "data_batch": b})
                while not self._stop.is_set():
                    try:
                        self.q.put(item, timeout=0.1)
                        break
                    except queue.Full:
                        continue
                if self._stop.is_set():
                    return
        except BaseException as e:  # surfaces in the consumer's next() instead of a silent stop
            self._error = e
        finally:
            self.q.put(None)

    def __iter__(self):
        return self

    def __next__(self):
        item = self.q.get()
        if item is None:
            if self._error is not None:
                raise RuntimeError("ImageNet loader thread failed") from self._error
            raise StopIteration
        packed, desc, labels, st = item
        self.epoch, self.cursor, self.batch_index = st["data_epoch"], st["data_cursor"], st["data_batch"]
        return packed, desc, labels

    def state(self):
        return {"data_epoch": self.epoch, "data_cursor": self.cursor, "data_batch": self.batch_index}

    def close(self):
        self._stop.set()
        try:
            while True:
                self.q.get_nowait()
        except queue.Empty:
            pass
        self._t.join(timeout=2)
        self.pool.shutdown(wait=self.workers == "process", cancel_futures=True)
        if self.workers == "process":
            _shm_cleanup(os.getpid())


def write_fake_imagenet(dirpath: str, shards: int = 2, per_shard: int = 8, is_training: bool = True,
                        seed: int = 0, num_classes: int = 1001) -> List[str]:
    """Writes small ImageNet-format TFRecord shards with random JPEGs (tests, smoke runs)."""
    from PIL import Image
    os.makedirs(dirpath, exist_ok=True)
    rng = np.random.default_rng(seed)
    out = []
    for s in range(shards):
        name = ("train-%05d-of-01024" if is_training else "validation-%05d-of-00128") % s
        path = os.path.join(dirpath, name)
        with TFRecordWriter(path) as w:
            for _ in range(per_shard):
                h, wd = int(rng.integers(200, 330)), int(rng.integers(200, 330))
                arr = rng.integers(0, 256, (h, wd, 3), dtype=np.uint8)
                b = io.BytesIO()
                Image.fromarray(arr).save(b, format="JPEG", quality=90)
                w.write(make_example(b.getvalue(), int(rng.integers(1, num_classes))))
        out.append(path)
    return out
