"""ctypes binding of the native host helper library (csrc/host/drn_host.cc -> libdrn_host.so).

CPU-only code (no GPU): CRC32C (SSE4.2), TFRecord framing scan and CIFAR record gathering.
A pure-Python fallback keeps every caller working when the library has not been built.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

_LIB = None
_TRIED = False
_LOCK = threading.Lock()
HOST_LIB = Path(__file__).resolve().parents[1] / "ops" / "libdrn_host.so"


def host_lib():
    global _LIB, _TRIED
    if _LIB is not None or _TRIED:
        return _LIB
    with _LOCK:
        if _TRIED:
            return _LIB
        _TRIED = True
        if not HOST_LIB.exists():
            try:
                from ..ops import build as _b
                _b.build_host(verbose=False)
            except Exception:  # pragma: no cover - toolchain missing
                return None
        try:
            h = ctypes.CDLL(str(HOST_LIB))
        except OSError:  # pragma: no cover
            return None
        h.drn_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        h.drn_crc32c.restype = ctypes.c_uint32
        h.drn_crc32c_masked.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        h.drn_crc32c_masked.restype = ctypes.c_uint32
        h.drn_tfrecord_scan.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_long, ctypes.c_int]
        h.drn_tfrecord_scan.restype = ctypes.c_long
        h.drn_cifar_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        h.drn_cifar_gather.restype = None
        _LIB = h
        return _LIB
