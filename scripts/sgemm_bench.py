#!/usr/bin/env python3
"""Microbenchmark of the head's fp32 GEMMs (ImageNet ResNet-50 dense layer, bs 128): logits,
dW and d(pooled), each timed over back-to-back launches and checked against torch.matmul.
usage: python scripts/sgemm_bench.py [--batch 128] [--classes 1001] [--features 2048]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_resnet_tensorflow_amd.ops.backend import HipBackend


def timeit(fn, iters=50):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--classes", type=int, default=1001)
    ap.add_argument("--features", type=int, default=2048)
    a = ap.parse_args()
    be = HipBackend()
    N, K, C = a.batch, a.classes, a.features
    torch.manual_seed(0)
    pooled = torch.randn(N, C, device="cuda")
    w = torch.randn(K, C, device="cuda") * 0.02
    b = torch.randn(K, device="cuda")
    dlog = torch.randn(N, K, device="cuda") * 0.01
    logits = torch.empty(N, K, device="cuda")
    dw = torch.empty(K, C, device="cuda")
    dpool = torch.empty(N, C, device="cuda")
    cases = [
        ("logits", lambda: be.sgemm(0, 1, N, K, C, 1.0, pooled, C, w, C, 0.0, logits, K, bias=b),
         lambda: pooled @ w.t() + b, logits, 2.0 * N * K * C),
        ("dW", lambda: be.sgemm(1, 0, K, C, N, 1.0, dlog, K, pooled, C, 0.0, dw, C),
         lambda: dlog.t() @ pooled, dw, 2.0 * N * K * C),
        ("dpool", lambda: be.sgemm(0, 0, N, C, K, 1.0, dlog, K, w, C, 0.0, dpool, C),
         lambda: dlog @ w, dpool, 2.0 * N * K * C),
    ]
    torch.backends.cuda.matmul.allow_tf32 = False
    for name, run, ref, out, fl in cases:
        t = timeit(run)
        run()
        torch.cuda.synchronize()
        r = ref()
        err = ((out - r).norm() / r.norm()).item()
        print(f"{name:7s} {t:8.1f} us  {fl / t / 1e6:7.1f} TF/s  rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
