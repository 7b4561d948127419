#!/usr/bin/env python3
"""What bounds the LDS-DMA convolution main loops? (isolate before tuning.)

The same kernels are built in four variants from a patched copy of the sources
(scripts/conv_bound_iso.patch; the shipped sources, and so the kernel database key, stay
unchanged), and a fixed set of ResNet-50 bs128 launches -- the in-step configurations of the
round-5 per-dispatch profile (profiles/r5_rn50_pmc_dispatch.txt) -- is timed under each:

  base    the real kernel
  noload  no LDS-DMA in the main loop (MFMA + fragment reads of whatever is in LDS)
  mfma    noload + no fragment reads either (operands are opaque registers): the matrix pipe alone
  nomfma  loads + fragment reads, no MFMA (operands kept live)
  noloop  no main loop at all: launch, prologue and epilogue (the fixed cost per tile)

    python scripts/conv_bound_iso.py --build          # CPU: gpu_variants/iso/<variant>/libdrn_kernels.so
    python scripts/conv_bound_iso.py --all [--out f]  # GPU: every variant (one process each), table
    DRN_KERNEL_LIB=... python scripts/conv_bound_iso.py --run [--case NAME]   # one library
"""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT_ROOT = os.path.join(REPO, "gpu_variants", "iso")
VARIANTS = {
    "base": [],
    "noload": ["-DDRN_ISO_NOLOAD"],
    "mfma": ["-DDRN_ISO_NOLOAD", "-DDRN_ISO_NOREAD"],
    "nomfma": ["-DDRN_ISO_NOMFMA"],
    "noloop": ["-DDRN_ISO_NOLOOP"],
}

# name: (kind, N, H(in), C, K(out), R, stride, pad, extra)
#   fwd extra: cfg (DRN conv config id), pro (fused BN-apply prologue), res (residual epilogue)
#   wgrad extra: ns (pipeline id), target (split-K block target)
CASES = {
    "fwd3x3_28": ("fwd", 128, 28, 128, 128, 3, 1, 1, dict(cfg=0)),
    "fwd3x3_14": ("fwd", 128, 14, 256, 256, 3, 1, 1, dict(cfg=0)),
    "fwd3x3_7": ("fwd", 128, 7, 512, 512, 3, 1, 1, dict(cfg=13)),
    "fwd1x1pro_56": ("fwd", 128, 56, 64, 256, 1, 1, 0, dict(cfg=13, pro=True, res=True)),
    "fwd1x1pro_14": ("fwd", 128, 14, 1024, 256, 1, 1, 0, dict(cfg=13, pro=True)),
    "fwd1x1_28": ("fwd", 128, 28, 128, 512, 1, 1, 0, dict(cfg=0, res=True)),
    "wgrad3x3_28": ("wgrad", 128, 28, 128, 128, 3, 1, 1, dict(ns=2, target=512)),
    "wgrad3x3_14": ("wgrad", 128, 14, 256, 256, 3, 1, 1, dict(ns=2, target=512)),
    "wgrad1x1_14": ("wgrad", 128, 14, 1024, 256, 1, 1, 0, dict(ns=2, target=512)),
    # the packed 7x7/2 stem's weight gradient (4-channel tap-pair layout, csrc/kernels/stem.hip):
    # input [N][224][226][4], taps 7 x 8 (the 8th tap zero), pad (3, 2); the last kernel of the step
    "fwd_stem": ("fwd", 128, 224, 4, 64, 7, 2, 3, dict(cfg=12, S=8, W=226, pad_w=2)),
    "wgrad_stem": ("wgrad", 128, 224, 4, 64, 7, 2, 3, dict(ns=2, target=512, S=8, W=226, pad_w=2)),
    # ... and by the input-halo kernel (conv_wgrad.hip stem_wgrad_halo_kernel, 3 / 4 stages)
    "wgrad_stem_halo3": ("wgrad", 128, 224, 4, 64, 7, 2, 3, dict(ns=9, target=512, S=8, W=226, pad_w=2)),
    "wgrad_stem_halo4": ("wgrad", 128, 224, 4, 64, 7, 2, 3, dict(ns=10, target=512, S=8, W=226, pad_w=2)),
    "wgrad_stem_halo3_768": ("wgrad", 128, 224, 4, 64, 7, 2, 3, dict(ns=9, target=768, S=8, W=226, pad_w=2)),
}
# --sweep: the 3x3 forward shapes under other tile / pipeline configurations (name@cfg)
SWEEP = {"fwd3x3_28": (1, 2, 8, 9, 17, 20, 27, 30, 31), "fwd3x3_14": (1, 2, 8, 9, 17, 20, 25, 26, 29, 30)}


def add_sweep():
    for name, cfgs in SWEEP.items():
        kind, N, H, C, K, R, st, pad, ex = CASES[name]
        for c in cfgs:
            CASES[f"{name}@{c}"] = (kind, N, H, C, K, R, st, pad, dict(ex, cfg=c))


def build(only=None):
    src = os.path.join(REPO, "build", "iso_src")
    shutil.rmtree(src, ignore_errors=True)
    os.makedirs(src)
    for d in ("kernels", "include"):
        shutil.copytree(os.path.join(REPO, "csrc", d), os.path.join(src, "csrc", d))
    subprocess.run(["patch", "-p0", "-s", "-i", os.path.join(REPO, "scripts", "conv_bound_iso.patch")], cwd=src,
                   check=True)
    from distributed_resnet_tensorflow_amd.ops.build import build_variant
    for name, flags in VARIANTS.items():
        if only and name not in only:
            continue
        lib = build_variant(os.path.join(OUT_ROOT, name), flags, src_root=os.path.join(src, "csrc"))
        print(f"[iso] built {name}: {lib}", flush=True)


def run(only=None, iters=50):
    import torch
    from distributed_resnet_tensorflow_amd.ops.backend import ConvGeom, HipBackend
    be = HipBackend()
    be.autotune = False
    st = be.stream()
    res = {}
    for name, (kind, N, H, C, K, R, stride, pad, ex) in CASES.items():
        if only and name not in only:
            continue
        S, W, pad_w = ex.get("S", R), ex.get("W", H), ex.get("pad_w", pad)
        P = (H + 2 * pad - R) // stride + 1
        x = torch.randn(N, H, W, C, device="cuda").bfloat16()
        g = ConvGeom(stride, pad, pad_w)
        flop = 2.0 * N * P * P * K * R * S * C
        if kind == "fwd":
            w = (torch.randn(K, R, S, C, device="cuda") * 0.05).bfloat16()
            y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
            in_bn = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1) if ex.get("pro") else None
            resid = torch.randn(N, P, P, K, device="cuda").bfloat16() if ex.get("res") else None
            a = be.conv_args(x, w, y, g, in_bn=in_bn, residual=resid)
            a.cfg = ex["cfg"]
            if be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), st) != 0:
                print(f"{name:14s} (configuration not applicable)", flush=True)
                continue
            fn = lambda: _lib_check(be.L.drn_conv_fwd2(ctypes.byref(a), be.zero_page.data_ptr(), st))
            nbytes = 2 * (x.numel() + w.numel() + y.numel() + (resid.numel() if resid is not None else 0))
        else:
            dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
            dw = torch.empty(K, R, S, C, device="cuda")
            ws = torch.empty(be.wgrad_ws_elems(N * P * P, K, R, S, C) or 1, device="cuda")
            a = be.wgrad_args(x, dy, dw, g, ws=ws, target_blocks=ex["target"])
            fn = lambda: _lib_check(be.L.drn_conv_wgrad2(ctypes.byref(a), be.zero_page.data_ptr(), ex["ns"], st))
            nbytes = 2 * (x.numel() + dy.numel()) + 4 * a.splits * dw.numel()
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(3):
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / iters * 1e3)
        res[name] = {"us": round(best, 2), "tflops": round(flop / best / 1e6, 1),
                     "gbs": round(nbytes / best / 1e3, 1)}
        print(f"{name:14s} {best:8.2f} us {flop / best / 1e6:7.1f} TF/s {nbytes / best / 1e3:7.1f} GB/s", flush=True)
    return res


def _lib_check(rc):
    if rc != 0:
        raise RuntimeError(f"launch refused (hipError {rc})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--case", action="append")
    ap.add_argument("--variant", action="append", help="--build / --all: only these variants")
    ap.add_argument("--sweep", action="store_true", help="also the 3x3 shapes under other configurations")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.sweep:
        add_sweep()
    if a.build:
        build(a.variant)
    if a.run:
        r = run(a.case, a.iters)
        if a.out:
            json.dump(r, open(a.out, "w"))
    if a.all:
        table = {}
        variants = [v for v in VARIANTS if not a.variant or v in a.variant]
        for name in variants:
            tmp = os.path.join(OUT_ROOT, f"{name}.json")
            env = dict(os.environ, DRN_KERNEL_LIB=os.path.join(OUT_ROOT, name, "libdrn_kernels.so"))
            cmd = [sys.executable, os.path.abspath(__file__), "--run", "--iters", str(a.iters), "--out", tmp]
            if a.sweep:
                cmd.append("--sweep")
            for c in a.case or []:
                cmd += ["--case", c]
            print(f"== {name}", flush=True)
            subprocess.run(cmd, env=env, check=True, timeout=600)
            table[name] = json.load(open(tmp))
        lines = ["# conv main-loop bound isolation (us per launch; TF/s of the real FLOPs)",
                 f"{'case':14s} " + " ".join(f"{v:>16s}" for v in variants)]
        for c in table[variants[0]]:
            lines.append(f"{c:14s} " + " ".join(
                f"{table[v][c]['us']:8.1f} {table[v][c]['tflops']:6.0f}T" if c in table[v] else f"{'-':>16s}"
                for v in variants))
        txt = "\n".join(lines)
        print(txt)
        if a.out:
            open(a.out, "w").write(txt + "\n" + json.dumps(table) + "\n")


if __name__ == "__main__":
    main()
