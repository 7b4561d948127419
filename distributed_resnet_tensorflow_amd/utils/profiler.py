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


def model_report(spec) -> str:
    lines = [f"model {spec.name}: {len(spec.trainable_variables())} trainable variables, "
             f"total_params: {spec.num_params():,}",
             f"forward GFLOP/image: {spec.forward_flops() / 1e9:.4f} "
             f"(train ~{3 * spec.forward_flops() / 1e9:.3f})"]
    return "\n".join(lines)
