#!/usr/bin/env python3
"""HBM roofline probes on the activation sizes of the ResNet-50 step: pure write (fill), copy,
and read-only (sum) of bf16 tensors."""
import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for n in (128 * 56 * 56 * 256, 128 * 56 * 56 * 64, 128 * 14 * 14 * 1024):
    a = torch.randn(n, device="cuda").bfloat16()
    b = torch.empty_like(a)
    nb = n * 2
    tf = timeit(lambda: b.fill_(1.0))
    tc = timeit(lambda: b.copy_(a))
    tr = timeit(lambda: a.sum(dtype=torch.float32))
    print(f"{nb / 1e6:7.1f} MB: fill {tf:6.1f} us ({nb / tf / 1e3:5.0f} GB/s)  copy {tc:6.1f} us "
          f"({2 * nb / tc / 1e3:5.0f} GB/s)  sum {tr:6.1f} us ({nb / tr / 1e3:5.0f} GB/s)", flush=True)
