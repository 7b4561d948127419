"""CRC32C (Castagnoli) and the TF/LevelDB "masked" CRC used by TFRecord, tfevents and
TensorBundle files. Native SSE4.2 implementation with a table-driven Python fallback."""
from __future__ import annotations

import ctypes

from .native import host_lib

_MASK_DELTA = 0xA282EAD8
_TABLE = []


def _py_table():
    if not _TABLE:
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            _TABLE.append(c)
    return _TABLE


def _as_buffer(data):
    if isinstance(data, (bytes, bytearray)):
        return data
    return memoryview(data).cast("B").tobytes()


def value(data, init: int = 0) -> int:
    lib = host_lib()
    if lib is not None:
        if isinstance(data, bytes):
            return lib.drn_crc32c(data, len(data), init)
        mv = memoryview(data).cast("B")
        if mv.readonly:
            b = mv.tobytes()
            return lib.drn_crc32c(b, len(b), init)
        buf = (ctypes.c_char * len(mv)).from_buffer(mv)
        return lib.drn_crc32c(ctypes.addressof(buf), len(mv), init)
    t = _py_table()
    crc = init ^ 0xFFFFFFFF
    for b in _as_buffer(data):
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def mask(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + _MASK_DELTA) & 0xFFFFFFFF


def unmask(masked: int) -> int:
    rot = (masked - _MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


def masked_value(data) -> int:
    return mask(value(data))
