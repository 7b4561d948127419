"""Minimal protocol-buffer wire-format encoder/decoder.

The reference writes TF protos (Event/Summary for TensorBoard, BundleHeaderProto /
BundleEntryProto for checkpoints, Example for ImageNet shards). TensorFlow is not available,
so the few messages needed are encoded field-by-field here; field numbers are documented at
each use site (events.py, ckpt/bundle.py, data/tfrecord.py).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

VARINT, I64, LEN, I32 = 0, 1, 2, 5


def varint(n: int) -> bytes:
    if n < 0:
        n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def tag(field: int, wt: int) -> bytes:
    return varint((field << 3) | wt)


def f_varint(field: int, v: int) -> bytes:
    return tag(field, VARINT) + varint(int(v))


def f_bytes(field: int, b: bytes) -> bytes:
    return tag(field, LEN) + varint(len(b)) + b


def f_string(field: int, s: str) -> bytes:
    return f_bytes(field, s.encode("utf-8"))


def f_double(field: int, v: float) -> bytes:
    return tag(field, I64) + struct.pack("<d", v)


def f_float(field: int, v: float) -> bytes:
    return tag(field, I32) + struct.pack("<f", v)


def f_fixed32(field: int, v: int) -> bytes:
    return tag(field, I32) + struct.pack("<I", v & 0xFFFFFFFF)


def read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def decode(buf: bytes) -> Dict[int, List]:
    """Field number -> list of raw values (int for varint/fixed, bytes for LEN)."""
    out: Dict[int, List] = {}
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = read_varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == VARINT:
            v, pos = read_varint(buf, pos)
        elif wt == I64:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == LEN:
            ln, pos = read_varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == I32:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(field, []).append(v)
    return out


def as_double(b: bytes) -> float:
    return struct.unpack("<d", b)[0]


def as_float(b: bytes) -> float:
    return struct.unpack("<f", b)[0]


def as_fixed32(b: bytes) -> int:
    return struct.unpack("<I", b)[0]


def signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v
