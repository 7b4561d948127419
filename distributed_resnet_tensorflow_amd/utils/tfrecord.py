"""TFRecord framing (used by ImageNet shards and tfevents files).

record := uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)
"""
from __future__ import annotations

import ctypes
import mmap
import os
import struct
from typing import Iterator, List, Tuple

import numpy as np

from . import crc32c
from .native import host_lib


def encode_record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", crc32c.masked_value(hdr)) + data + struct.pack("<I", crc32c.masked_value(data))


class TFRecordWriter:
    def __init__(self, path: str):
        self.path = path
        self.f = open(path, "ab")

    def write(self, data: bytes):
        self.f.write(encode_record(data))

    def flush(self):
        self.f.flush()
        os.fsync(self.f.fileno())

    def close(self):
        if self.f:
            self.f.flush()
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class CorruptRecordError(IOError):
    pass


def scan(buf, check: bool = True) -> List[Tuple[int, int]]:
    """(offset, length) of every record in a TFRecord byte buffer, CRC-checked."""
    lib = host_lib()
    n = len(buf)
    if lib is not None and n > 0:
        cap = max(16, n // 16)
        offs = np.zeros(cap, dtype=np.int64)
        lens = np.zeros(cap, dtype=np.int64)
        mv = memoryview(buf)
        if mv.readonly:
            raw = bytes(mv)
            ptr = ctypes.cast(ctypes.c_char_p(raw), ctypes.c_void_p).value
        else:
            carr = (ctypes.c_char * n).from_buffer(mv)
            ptr = ctypes.addressof(carr)
        cnt = lib.drn_tfrecord_scan(ptr, n, offs.ctypes.data, lens.ctypes.data, cap, 1 if check else 0)
        if cnt < 0:
            raise CorruptRecordError(f"corrupt TFRecord at record {-cnt - 1}")
        return list(zip(offs[:cnt].tolist(), lens[:cnt].tolist()))
    out, pos = [], 0
    while pos + 12 <= n:
        (ln,) = struct.unpack_from("<Q", buf, pos)
        if check:
            (lc,) = struct.unpack_from("<I", buf, pos + 8)
            if crc32c.masked_value(bytes(buf[pos:pos + 8])) != lc:
                raise CorruptRecordError(f"bad length crc at byte {pos}")
            (dc,) = struct.unpack_from("<I", buf, pos + 12 + ln)
            if crc32c.masked_value(bytes(buf[pos + 12:pos + 12 + ln])) != dc:
                raise CorruptRecordError(f"bad data crc at byte {pos}")
        out.append((pos + 12, ln))
        pos += 12 + ln + 4
    return out


def read_records(path: str, check: bool = True) -> Iterator[bytes]:
    size = os.path.getsize(path)
    if size == 0:
        return
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as mm:
        data = bytes(mm)
    for off, ln in scan(data, check):
        yield data[off:off + ln]
