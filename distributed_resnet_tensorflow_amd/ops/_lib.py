"""Loader for the in-tree gfx950 kernel library ``libdrn_kernels.so`` (ctypes, C ABI).

The GPU compute path of this framework IS this library: there is no silent fallback. When a
GPU is present and the library is missing or fails to load, :func:`lib` raises. The CPU
reference backend (``ops.ref``) exists only for CPU-only runs (BASELINE config 1) and as the
fp32 test oracle.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must be imported first: its HIP runtime is the one we bind to)

_LIB = None
_LOCK = threading.Lock()
LIB_PATH = Path(os.environ.get("DRN_KERNEL_LIB") or Path(__file__).resolve().parent / "libdrn_kernels.so")
# diagnostics-only entry points an older library (A/B runs via DRN_KERNEL_LIB) may lack
_OPTIONAL = {"drn_conv_trace_set", "drn_wgrad_trace_set"}  # a -DDRN_CONV_TRACE build only

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_f = ctypes.c_float
c_p = ctypes.c_void_p


class DrnFastDiv(ctypes.Structure):
    _fields_ = [("d", ctypes.c_uint32), ("m", ctypes.c_uint32), ("s", ctypes.c_uint32), ("pad_", ctypes.c_uint32)]

    @classmethod
    def make(cls, d: int) -> "DrnFastDiv":
        d = int(max(1, d))
        s = 0
        while (1 << s) < d:
            s += 1
        m = ((1 << 32) * ((1 << s) - d)) // d + 1
        return cls(d, m & 0xFFFFFFFF, s, 0)


class DrnBnFin(ctypes.Structure):
    """Mirror of csrc/include/drn_conv.h `struct DrnBnFin` (consumer-side BatchNorm finalize)."""
    _fields_ = [
        ("stats", c_p), ("gamma", c_p), ("beta", c_p), ("run_mean", c_p), ("run_var", c_p), ("scale", c_p),
        ("shift", c_p), ("mean", c_p), ("invstd", c_p), ("dgamma", c_p), ("dbeta", c_p),
        ("G", c_int), ("C", c_int), ("count", c_f), ("eps", c_f), ("momentum", c_f), ("publish", c_int),
    ]


class DrnConvFwdArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_p), ("w", c_p), ("y", c_p), ("in_scale", c_p), ("in_shift", c_p), ("residual", c_p), ("stats", c_p),
        ("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("K", c_int), ("R", c_int), ("S", c_int),
        ("P", c_int), ("Q", c_int), ("stride", c_int), ("pad_h", c_int), ("pad_w", c_int), ("dil", c_int),
        ("relu_in", c_int), ("tiles_p", c_int),
        ("out_H", c_int), ("out_W", c_int), ("out_stride", c_int), ("out_oh", c_int), ("out_ow", c_int),
        ("cfg", c_int), ("stats_rep", c_int),
        ("bn_x", c_p), ("bn_scale", c_p), ("bn_shift", c_p), ("bn_mean", c_p), ("bn_invstd", c_p),
        ("fin_cnt", c_p), ("fin_count", ctypes.c_float), ("fin_eps", ctypes.c_float),
        ("fin_momentum", ctypes.c_float), ("out_fill", c_int),
        ("fin_gamma", c_p), ("fin_beta", c_p), ("fin_run_mean", c_p), ("fin_run_var", c_p),
        ("fin_scale", c_p), ("fin_shift", c_p), ("fin_mean", c_p), ("fin_invstd", c_p),
        ("fin_dgamma", c_p), ("fin_dbeta", c_p), ("fin_coef", c_p),
        ("fd_pq", DrnFastDiv), ("fd_q", DrnFastDiv), ("in_fin", DrnBnFin),
        ("ks_ws", c_p), ("ks_tickets", c_p), ("ksplit", c_int), ("sk_blocks", c_int),
    ]


class DrnConvWgradArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_p), ("dy", c_p), ("out", c_p), ("in_scale", c_p), ("in_shift", c_p),
        ("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("K", c_int), ("R", c_int), ("S", c_int),
        ("P", c_int), ("Q", c_int), ("stride", c_int), ("pad_h", c_int), ("pad_w", c_int), ("relu_in", c_int),
        ("splits", c_int), ("pix_per_split", c_int), ("fd_pq", DrnFastDiv), ("fd_q", DrnFastDiv),
        ("atomic_out", c_int),
    ]


_SIGS = {
    "drn_version": ([], c_int),
    "drn_conv_fwd": ([ctypes.POINTER(DrnConvFwdArgs), c_p], c_int),
    "drn_conv_fwd_tiles_p": ([c_int, c_int], c_int),
    "drn_conv_fwd2": ([ctypes.POINTER(DrnConvFwdArgs), c_p, c_p], c_int),
    "drn_conv_glds_ok": ([ctypes.POINTER(DrnConvFwdArgs)], c_int),
    "drn_conv_glds_num_cfgs": ([], c_int),
    "drn_conv_trace_set": ([c_p], c_int),
    "drn_wgrad_trace_set": ([c_p], c_int),
    "drn_conv_glds_default_cfg": ([ctypes.POINTER(DrnConvFwdArgs)], c_int),
    "drn_conv_wgrad": ([ctypes.POINTER(DrnConvWgradArgs), c_p], c_int),
    "drn_conv_wgrad2": ([ctypes.POINTER(DrnConvWgradArgs), c_p, c_int, c_p], c_int),
    "drn_splitk_reduce": ([c_p, c_p, c_i64, c_int, c_f, c_int, c_p], c_int),
    "drn_bn_stats": ([c_p, c_p, c_int, c_int, c_int, c_int, c_p], c_int),
    "drn_bn_finalize": ([c_p, c_int, c_int, c_f, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_int),
    "drn_bn_inference_params": ([c_int, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p], c_int),
    "drn_bn_apply": ([c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_p], c_int),
    "drn_bn_apply_stats": ([c_p, c_p, c_p, c_f, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_int,
                            c_int, c_p], c_int),
    "drn_bn_bwd_apply_stats": ([c_p, c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_i64,
                                c_int, c_int, c_p], c_int),
    "drn_bn_bwd_reduce": ([c_p, c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p],
                          c_int),
    "drn_bn_finalize_bwd": ([c_p, c_int, c_int, c_f, c_p, c_p, c_p, c_p, c_p, c_p], c_int),
    "drn_bn_bwd_apply": ([c_p, c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_p], c_int),
    "drn_bnrelu_pool": ([c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p], c_int),
    "drn_sgemm": ([c_int, c_int, c_int, c_int, c_int, c_f, c_p, c_int, c_p, c_int, c_f, c_p, c_int, c_p, c_int, c_p,
                   c_p], c_int),
    "drn_softmax_xent": ([c_p, c_p, c_int, c_int, c_f, c_p, c_p, c_p, c_p, c_p], c_int),
    "drn_colsum": ([c_p, c_int, c_int, c_p, c_f, c_int, c_p], c_int),
    "drn_maxpool_fwd": ([c_p, c_p, c_p] + [c_int] * 10 + [c_p, c_int, c_p], c_int),
    "drn_maxpool_bwd": ([c_p, c_p, c_p] + [c_int] * 10 + [c_p], c_int),
    "drn_sgd_momentum": ([c_p, c_p, c_p, c_int, c_p, c_i64, c_p, c_f, c_f, c_f, c_p, c_p], c_int),
    "drn_cast_bf16": ([c_p, c_p, c_i64, c_p], c_int),
    "drn_stem_pack_input": ([c_p, c_p, c_int, c_int, c_p], c_int),
    "drn_stem_pack_weights": ([c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p], c_int),
    "drn_stem_unpack_grad": ([c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p], c_int),
    "drn_stem_conv_pool": ([c_p, c_p, c_p, c_p, c_p] + [c_int] * 11 + [c_p], c_int),
    "drn_weight_tflip": ([c_p, c_p, c_p, c_int, c_i64, c_p], c_int),
    "drn_fill_f32": ([c_p, c_i64, c_f, c_p], c_int),
    "drn_cifar_augment": ([c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p], c_int),
    "drn_vgg_preprocess": ([c_p, c_p, c_p, c_int, c_int, c_int, c_f, c_f, c_f, c_p], c_int),
    "drn_p2p_signal": ([c_p, c_int, c_p], c_int),
    "drn_p2p_reduce": ([c_p, c_int, c_int, c_p], c_int),
    "drn_p2p_reduce2": ([c_p, c_int, c_int, c_p], c_int),
    "drn_p2p_step": ([c_p, c_p, c_p], c_int),
    "drn_p2p_cast": ([c_p, c_p, c_i64, c_p], c_int),
    "drn_p2p_args_size": ([], c_int),
    "drn_conv_glds_cfg_bc": ([c_int], c_int),
    "drn_conv_glds_cfg_bp": ([c_int], c_int),
    "drn_conv_glds_cfg_bk": ([c_int], c_int),
    "drn_conv_sk_slots_cfg": ([c_p, c_int, c_int], c_int),
    "drn_conv_nk_num_cfgs": ([], c_int),
    "drn_conv_nk_cfg0": ([], c_int),
    "drn_p2p_alloc": ([ctypes.POINTER(c_p), ctypes.c_size_t], c_int),
    "drn_p2p_free": ([c_p], c_int),
    "drn_bn_fin_size": ([], c_int),
    "drn_conv_args_size": ([], c_int),
    "drn_wgrad_args_size": ([], c_int),
    "drn_bn_fin_fwd_launch": ([c_p, c_p], c_int),
    "drn_bn_apply_fin": ([c_p, c_p, c_p, c_i64, c_int, c_int, c_p], c_int),
    "drn_bn_bwd_apply_fin": ([c_p, c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_p], c_int),
    "drn_synthetic_images": ([c_p, c_i64, ctypes.c_uint32, c_p], c_int),
    # native step plans (csrc/kernels/plan.hip, runtime/plan.py)
    "drn_plan_create": ([], c_p),
    "drn_plan_destroy": ([c_p], None),
    "drn_plan_record_begin": ([c_p], c_int),
    "drn_plan_record_end": ([], c_int),
    "drn_plan_new_event": ([c_p], c_int),
    "drn_plan_event_record": ([c_p, c_int, c_p], c_int),
    "drn_plan_stream_wait": ([c_p, c_p, c_int], c_int),
    "drn_plan_size": ([c_p], c_int),
    "drn_plan_launches": ([c_p], c_int),
    "drn_plan_replay": ([c_p, c_int, c_int], c_int),
    "drn_plan_set_threads": ([c_p, c_int], c_int),
    "drn_plan_lanes": ([c_p], c_int),
    "drn_plan_count": ([c_p, c_int], c_int),
    "drn_plan_live_records": ([c_p], c_int),
}


class KernelLibraryError(RuntimeError):
    pass


def available() -> bool:
    return LIB_PATH.exists()


def lib():
    """Load (once) and return the kernel library; raise if it is missing or broken."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not LIB_PATH.exists():
            if os.environ.get("DRN_AUTOBUILD", "1") == "1":
                from . import build as _build
                _build.build(verbose=False)
            if not LIB_PATH.exists():
                raise KernelLibraryError(
                    f"{LIB_PATH} is missing: build it with `python -m distributed_resnet_tensorflow_amd.ops.build`")
        try:
            h = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover
            raise KernelLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (args, res) in _SIGS.items():
            if name in _OPTIONAL and not hasattr(h, name):
                continue
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        for name, st in (("drn_bn_fin_size", DrnBnFin), ("drn_conv_args_size", DrnConvFwdArgs),
                         ("drn_wgrad_args_size", DrnConvWgradArgs)):
            if getattr(h, name)() != ctypes.sizeof(st):
                raise KernelLibraryError(f"{st.__name__} layout mismatch between Python and {LIB_PATH.name}")
        _check_stamp(h)
        _LIB = h
        return _LIB


def _check_stamp(h) -> None:
    """Refuse a library built from other kernel sources than the tree's (source hash compiled in by
    ops.build); skipped when the sources are absent (an installed library) or for an explicit
    A/B library (DRN_KERNEL_LIB)."""
    from . import build as _build
    if os.environ.get("DRN_KERNEL_LIB") or not any(_build.KERNELS.glob("*.hip")):
        return
    if not hasattr(h, "drn_src_hash"):
        raise KernelLibraryError(f"{LIB_PATH} has no source stamp: rebuild it (python -m "
                                 "distributed_resnet_tensorflow_amd.ops.build)")
    h.drn_src_hash.restype = ctypes.c_char_p
    h.drn_src_hash.argtypes = []
    built = h.drn_src_hash().decode()
    want = _build.source_hash()
    if built != want:
        raise KernelLibraryError(f"{LIB_PATH} was built from different kernel sources (stamp {built[:12]}, tree "
                                 f"{want[:12]}): rebuild it (python -m distributed_resnet_tensorflow_amd.ops.build)")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise KernelLibraryError(f"{what} failed with hipError {rc}")
