"""TensorBoard event-file writer/reader (tensorboard is not installed; self-built).

Replaces TF's FileWriter / SummarySaverHook output (reference resnet_cifar_main.py:274-278,
resnet_cifar_eval.py:93, :125-136): `events.out.tfevents.<time>.<host>` files of TFRecord-framed
`Event` protos.
  Event   { double wall_time = 1; int64 step = 2; string file_version = 3; Summary summary = 5; }
  Summary { repeated Value value = 1; }
  Value   { string tag = 1; float simple_value = 2; Image image = 4; }
  Image   { int32 height = 1; int32 width = 2; int32 colorspace = 3; bytes encoded_image_string = 4; }
"""
from __future__ import annotations

import io
import os
import socket
import threading
import time
from typing import Dict, Iterator, List, Optional, Tuple

from . import pbwire as pb
from .tfrecord import TFRecordWriter, read_records


def _event(step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None,
           wall_time: Optional[float] = None) -> bytes:
    b = pb.f_double(1, time.time() if wall_time is None else wall_time) + pb.f_varint(2, step)
    if file_version is not None:
        b += pb.f_string(3, file_version)
    if summary is not None:
        b += pb.f_bytes(5, summary)
    return b


def scalar_value(tag: str, v: float) -> bytes:
    return pb.f_bytes(1, pb.f_string(1, tag) + pb.f_float(2, float(v)))


def image_value(tag: str, png: bytes, h: int, w: int, c: int) -> bytes:
    img = pb.f_varint(1, h) + pb.f_varint(2, w) + pb.f_varint(3, c) + pb.f_bytes(4, png)
    return pb.f_bytes(1, pb.f_string(1, tag) + pb.f_bytes(4, img))


def encode_png(img_u8) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(img_u8).save(buf, format="PNG")
    return buf.getvalue()


class EventFileWriter:
    """Append-only tfevents writer; thread-safe, flushed every `flush_secs`."""

    def __init__(self, logdir: str, flush_secs: float = 10.0, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        fname = f"events.out.tfevents.{int(time.time()):010d}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(logdir, fname)
        self._w = TFRecordWriter(self.path)
        self._lock = threading.Lock()
        self._last_flush = time.time()
        self.flush_secs = flush_secs
        self._w.write(_event(0, file_version="brain.Event:2"))
        self.flush()

    def add_scalars(self, step: int, scalars: Dict[str, float]):
        summ = b"".join(scalar_value(k, v) for k, v in scalars.items())
        self._write(_event(int(step), summary=summ))

    def add_scalar(self, tag: str, value: float, step: int):
        self.add_scalars(step, {tag: value})

    def add_images(self, step: int, tag: str, images_u8, max_images: int = 3):
        vals = []
        for i, im in enumerate(images_u8[:max_images]):
            h, w = im.shape[:2]
            c = im.shape[2] if im.ndim == 3 else 1
            vals.append(image_value(f"{tag}/image/{i}" if max_images > 1 else f"{tag}/image", encode_png(im), h, w, c))
        self._write(_event(int(step), summary=b"".join(vals)))

    def _write(self, ev: bytes):
        with self._lock:
            self._w.write(ev)
            if time.time() - self._last_flush > self.flush_secs:
                self._w.f.flush()
                self._last_flush = time.time()

    def flush(self):
        with self._lock:
            self._w.f.flush()
            self._last_flush = time.time()

    def close(self):
        with self._lock:
            self._w.close()


def read_events(path: str) -> Iterator[Tuple[float, int, Dict[str, float]]]:
    """Yields (wall_time, step, {tag: simple_value}) for every Event with scalar summaries."""
    for rec in read_records(path):
        f = pb.decode(rec)
        wall = pb.as_double(f[1][0]) if 1 in f else 0.0
        step = pb.signed64(f[2][0]) if 2 in f else 0
        scal = {}
        for s in f.get(5, []):
            for v in pb.decode(s).get(1, []):
                vf = pb.decode(v)
                tag = vf[1][0].decode() if 1 in vf else ""
                if 2 in vf:
                    scal[tag] = pb.as_float(vf[2][0])
                elif 4 in vf:
                    scal[tag] = float("nan")
        yield wall, step, scal


def scalar_series(logdir: str, tag: str) -> List[Tuple[int, float]]:
    out = []
    for fn in sorted(os.listdir(logdir)):
        if fn.startswith("events.out.tfevents"):
            for _, step, sc in read_events(os.path.join(logdir, fn)):
                if tag in sc:
                    out.append((step, sc[tag]))
    return out
