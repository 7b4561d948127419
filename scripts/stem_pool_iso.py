#!/usr/bin/env python3
"""Isolated time of the ImageNet stem forward at bs 128: the fused conv + max-pool kernel
(csrc/kernels/stem_pool.hip) vs the two-kernel path (packed conv with the tuned configuration,
then maxpool_fwd), both with the pooled BN statistics; best of 3 x 50 launches.

    python scripts/stem_pool_iso.py [--batch 128]
    python scripts/stem_pool_iso.py --build-variants   (on the build host: gpu_variants/stem/*)
    python scripts/stem_pool_iso.py --variants          (on the GPU: each variant's fused time)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend  # noqa: E402


def best_us(fn, n=50, rounds=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--build-variants", action="store_true")
    ap.add_argument("--variants", action="store_true")
    ap.add_argument("--fused-only", action="store_true")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = ("NOLOAD", "NOMMA", "NOPOOL")
    if a.build_variants:
        from distributed_resnet_tensorflow_amd.ops import build
        for v in names:
            print(build.build_variant(os.path.join(root, "gpu_variants", "stem", v.lower()), [f"-DDRN_STEM_ISO_{v}"]))
        return
    if a.variants:
        import subprocess
        for v in ("base",) + names:
            env = dict(os.environ)
            if v != "base":
                env["DRN_KERNEL_LIB"] = os.path.join(root, "gpu_variants", "stem", v.lower(), "libdrn_kernels.so")
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--fused-only", "--batch", str(a.batch)],
                                 capture_output=True, text=True, env=env, timeout=120)
            print(f"{v:>7}: {out.stdout.strip() or out.stderr[-300:]}", flush=True)
        return
    be = HipBackend("cuda")
    N, H, K, pad = a.batch, 224, 64, 3
    P = (H + 2 * pad - 7) // 2 + 1
    PP = (P + 1) // 2
    xp = torch.randn(N, H, H + 2, 4, device="cuda").bfloat16()
    xp[:, :, 0] = 0
    xp[:, :, H + 1] = 0
    w4 = (torch.randn(K, 7, 8, 4, device="cuda") * 0.1).bfloat16()
    w4[:, :, 7] = 0
    g4 = ConvGeom(stride=2, pad_h=pad, pad_w=pad - 1)
    y = torch.empty(N, P, P, K, dtype=torch.bfloat16, device="cuda")
    yp = torch.empty(N, PP, PP, K, dtype=torch.bfloat16, device="cuda")
    arg = torch.empty(N, PP, PP, K, dtype=torch.uint8, device="cuda")
    st = torch.zeros(8, 2, K, device="cuda")

    def two():
        be.conv_fwd(xp, w4, y, g4)
        be.maxpool_fwd(y, yp, arg, 3, 2, 0, 0, stats=st)

    def fused():
        be.stem_conv_pool(xp, w4, yp, arg, g4, H, H, P, P, stats=st)

    if a.fused_only:
        print(f"fused {best_us(fused):.1f} us")
        return
    t_conv = best_us(lambda: be.conv_fwd(xp, w4, y, g4))
    t_pool = best_us(lambda: be.maxpool_fwd(y, yp, arg, 3, 2, 0, 0, stats=st))
    t_two, t_fused = best_us(two), best_us(fused)
    mb = (N * H * (H + 2) * 8 + N * PP * PP * K * 3) / 1e6
    print(f"bs {N}: conv {t_conv:.1f} us + maxpool {t_pool:.1f} us = two-kernel {t_two:.1f} us; "
          f"fused {t_fused:.1f} us ({mb / t_fused:.2f} TB/s of compulsory {mb:.0f} MB)", flush=True)


if __name__ == "__main__":
    main()
