"""roctx markers (librocprofiler-sdk-roctx) for rocprofv3 --marker-trace, and the tfprof-style
parameter/FLOP report (reference resnet_single.py:58-66 printed trainable params + FLOPs)."""
from __future__ import annotations

import ctypes
import ctypes.util


class Roctx:
    def __init__(self):
        self.lib = None
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
            try:
                self.lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if self.lib is not None:
            self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            self.lib.roctxRangePushA.restype = ctypes.c_int
            self.lib.roctxRangePop.restype = ctypes.c_int

    def push(self, msg: str):
        if self.lib is not None:
            self.lib.roctxRangePushA(msg.encode())

    def pop(self):
        if self.lib is not None:
            self.lib.roctxRangePop()


_ROCTX = None
_PHASES_ON = False


def enable_phases(on: bool = True) -> None:
    """Turn the per-step phase ranges on (ProfileHook / DRN_ROCTX=1). Off, phase() costs one
    attribute check."""
    global _ROCTX, _PHASES_ON
    if on and _ROCTX is None:
        _ROCTX = Roctx()
    _PHASES_ON = bool(on) and _ROCTX is not None and _ROCTX.lib is not None


class phase:
    """`with phase("fwd"):` -- a roctx range (rocprofv3 --marker-trace) around one phase of the
    training step (data / fwd / bwd / comm / optimizer). Host-side ranges: they
    bracket the enqueue of the phase's kernels (for device time, pair them with --kernel-trace)."""
    __slots__ = ("name", "on")

    def __init__(self, name: str):
        self.name = name
        self.on = _PHASES_ON

    def __enter__(self):
        if self.on:
            _ROCTX.push(self.name)
        return self

    def __exit__(self, *exc):
        if self.on:
            _ROCTX.pop()
        return False


def model_report(spec) -> str:
    lines = [f"model {spec.name}: {len(spec.trainable_variables())} trainable variables, "
             f"total_params: {spec.num_params():,}",
             f"forward GFLOP/image: {spec.forward_flops() / 1e9:.4f} "
             f"(train ~{3 * spec.forward_flops() / 1e9:.3f})"]
    return "\n".join(lines)
