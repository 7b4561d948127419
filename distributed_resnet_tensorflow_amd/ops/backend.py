"""Compute backends behind the static-plan executor.

``HipBackend`` is THE training path on MI355X: every call is one launch of a hand-written
gfx950 kernel from ``libdrn_kernels.so`` on the current HIP stream (ctypes, raw device
pointers — capturable into a HIP graph). ``RefBackend`` implements the identical op contract
in fp32 PyTorch on the CPU; it is used for CPU-only runs (BASELINE config 1, the reference's
`--num_gpus=0` CPU mode, resnet_cifar_main.py:387-390) and as the numerics oracle in tests.
No op silently falls back from one to the other.

Op contract (NHWC activations, KRSC conv weights, fp32 statistics):
  conv_fwd(x, w, y, g, in_bn, relu_in, residual, stats)      y = conv(pre(x), w) [+ residual]
  conv_wgrad(x, dy, out, g, in_bn, relu_in, ws, splits)      out = dW (fp32, KRSC)
  bn_stats / bn_finalize / bn_inference / bn_apply
  bn_bwd_reduce / bn_finalize_bwd / bn_bwd_apply
  pool_bnrelu, sgemm, softmax_xent, colsum, maxpool_fwd/bwd, sgd_momentum, weight_tflip
where pre(x) = relu(x * scale + shift) when in_bn = (scale, shift) is given.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib


@dataclass(frozen=True)
class ConvGeom:
    """Geometry of one convolution launch (forward, or data-gradient as a forward conv)."""
    stride: int = 1
    pad_h: int = 0
    pad_w: int = 0
    dil: int = 1  # 2: zero-dilated (transposed) input, used for stride-2 data gradients


def _ptr(t):
    return None if t is None else t.data_ptr()


def dgrad_geom(g: ConvGeom, R: int, S: int) -> ConvGeom:
    """Data-gradient of a forward conv (stride s, leading pad p) as a forward conv of dY with the
    flipped, channel-transposed weights: stride 1, leading pad k-1-p, input dilated by s."""
    return ConvGeom(stride=1, pad_h=R - 1 - g.pad_h, pad_w=S - 1 - g.pad_w, dil=g.stride)


TDESC = np.dtype([("src", "<i8"), ("dst", "<i8"), ("K", "<i4"), ("R", "<i4"), ("S", "<i4"), ("C", "<i4"),
                  ("Ru", "<i4"), ("Sv", "<i4"), ("r0", "<i4"), ("s0", "<i4"), ("dr", "<i4"), ("ds", "<i4"),
                  ("tk", "<i4"), ("tc", "<i4"), ("begin", "<i8")])  # mirror of sgd.hip `struct TDesc`


def tflip_desc(src, dst, K, R, S, C, Ru=None, Sv=None, r0=None, s0=None, dr=-1, ds=-1):
    """Dgrad weight extraction Wt[c][u][v][k] = W[k][r0+dr*u][s0+ds*v][c]; defaults = full flip."""
    Ru = R if Ru is None else Ru
    Sv = S if Sv is None else Sv
    r0 = R - 1 if r0 is None else r0
    s0 = S - 1 if s0 is None else s0
    return (src, dst, K, R, S, C, Ru, Sv, r0, s0, dr, ds)


def tflip_table(descs):
    """Pack descriptors (see tflip_desc) into the byte table of drn_weight_tflip: the kernel is a
    tiled transpose with one workgroup per (descriptor, tap, 64 k, 64 c) tile; `begin` is the
    tile prefix sum and the returned total is the tile count (= the launch grid)."""
    arr = np.zeros(max(1, len(descs)), dtype=TDESC)
    begin = 0
    for i, d in enumerate(descs):
        src, dst, K, R, S, C, Ru, Sv, r0, s0, dr, ds = d
        if K % 8 or C % 8:
            raise ValueError(f"weight_tflip needs K and C multiples of 8 (got K={K}, C={C})")
        tk, tc = -(-K // 64), -(-C // 64)
        arr[i] = (src, dst, K, R, S, C, Ru, Sv, r0, s0, dr, ds, tk, tc, begin)
        begin += Ru * Sv * tk * tc
    return torch.from_numpy(arr.view(np.uint8).copy()), len(descs), begin


def _aligned16(*ts):
    """The fused BN kernels read per-channel vectors with 16-byte loads."""
    for t in ts:
        if t is not None and t.data_ptr() % 16:
            raise ValueError("per-channel BN buffers must be 16-byte aligned")


@dataclass
class BnFin:
    """BatchNorm finalize fused into the convolution producing its statistics (the last-arriving
    workgroup of each channel column; DrnConvFwdArgs.fin_cnt). Forward (no bn_bwd): scale/shift/
    mean/invstd + moving averages from the sums; backward (with bn_bwd): dgamma, dbeta and the
    apply coefficients coef[3][C]."""
    counters: torch.Tensor            # int32, >= C/64 zeroed words (re-armed by the kernel)
    count: float                      # rows N*H*W of the normalised tensor
    gamma: torch.Tensor
    beta: Optional[torch.Tensor] = None
    run_mean: Optional[torch.Tensor] = None
    run_var: Optional[torch.Tensor] = None
    scale: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    mean: Optional[torch.Tensor] = None
    invstd: Optional[torch.Tensor] = None
    dgamma: Optional[torch.Tensor] = None
    dbeta: Optional[torch.Tensor] = None
    coef: Optional[torch.Tensor] = None
    momentum: float = 0.997
    eps: float = 1e-5


@dataclass
class BnCfin:
    """Consumer-side BatchNorm finalize (csrc/include/drn_conv.h DrnBnFin): the kernel that
    CONSUMES a BatchNorm derives its parameters from the statistics replicas `stats` [G][2][C]
    in its own prologue instead of a separate finalize launch; with `publish` its first workgroup
    also writes them out (forward: scale/shift/mean/invstd + moving averages; backward: dgamma,
    dbeta) for the kernels that run later."""
    stats: torch.Tensor
    count: float
    gamma: torch.Tensor
    beta: Optional[torch.Tensor] = None
    run_mean: Optional[torch.Tensor] = None
    run_var: Optional[torch.Tensor] = None
    scale: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    mean: Optional[torch.Tensor] = None
    invstd: Optional[torch.Tensor] = None
    dgamma: Optional[torch.Tensor] = None
    dbeta: Optional[torch.Tensor] = None
    publish: bool = False
    momentum: float = 0.997
    eps: float = 1e-5

    @property
    def C(self) -> int:
        return self.gamma.numel()

    @property
    def G(self) -> int:
        return self.stats.numel() // (2 * self.C)

    def struct(self):
        f = _lib.DrnBnFin()
        f.stats, f.gamma, f.beta = self.stats.data_ptr(), self.gamma.data_ptr(), _ptr(self.beta)
        f.run_mean, f.run_var = _ptr(self.run_mean), _ptr(self.run_var)
        f.scale, f.shift, f.mean, f.invstd = _ptr(self.scale), _ptr(self.shift), _ptr(self.mean), _ptr(self.invstd)
        f.dgamma, f.dbeta = _ptr(self.dgamma), _ptr(self.dbeta)
        f.G, f.C = self.G, self.C
        f.count, f.eps, f.momentum = float(self.count), float(self.eps), float(self.momentum)
        f.publish = 1 if self.publish else 0
        return f


@dataclass(frozen=True)
class OutMap:
    """Strided output mapping of a phase of a stride-2 data gradient: the GEMM's P x Q grid lands
    at y[:, i*stride + oh, j*stride + ow, :] of the full output tensor."""
    P: int
    Q: int
    stride: int
    oh: int
    ow: int


# ----------------------------------------------------------------------------------------------
# HIP backend
# ----------------------------------------------------------------------------------------------
class _Common:
    @staticmethod
    def bn_stats_blocks(M, C):
        """Rows of a BN statistics accumulator: always 1 ([2][C] accumulated in place)."""
        return 1

    @staticmethod
    def conv_stats_tiles(M, K):
        return 1

    # Finalize fused into the apply kernels (HIP overrides with single kernels). Contract: the
    # statistics accumulator is left unchanged (the executor clears its arena per step).
    def bn_apply_stats(self, x, y, acc, count, gamma, beta, run_mean, run_var, scale, shift, mean, invstd,
                       momentum, eps, relu=True):
        self.bn_finalize(acc.clone(), 1, count, gamma, beta, run_mean, run_var, scale, shift, mean, invstd,
                         momentum, eps, update_running=True)
        self.bn_apply(x, y, scale, shift, relu=relu)

    def bn_bwd_apply_stats(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, acc, count, gamma, dgamma,
                           dbeta, add, dx, coef, relu=True):
        self.bn_finalize_bwd(acc.clone(), 1, count, gamma, invstd, dgamma, dbeta, coef)
        self.bn_bwd_apply(dy, dpool, pool_hw, x, scale, shift, mean, invstd, coef, add, dx, relu=relu)


    def fill_(self, t, v: float):
        t.fill_(v)

    # Consumer-side finalize (BnCfin) composed from the separate ops; HIP overrides with kernels
    # that finalize in their prologue.
    def _publish_fwd(self, f: BnCfin):
        self.bn_finalize(f.stats, f.G, f.count, f.gamma, f.beta, f.run_mean, f.run_var, f.scale, f.shift, f.mean,
                         f.invstd, f.momentum, f.eps, update_running=f.run_mean is not None)

    def bn_apply_fin(self, x, y, fin: BnCfin, relu=True):
        if fin.publish:
            self._publish_fwd(fin)
        self.bn_apply(x, y, fin.scale, fin.shift, relu=relu)

    def bn_bwd_apply_fin(self, dy, dpool, pool_hw, x, scale, shift, fin: BnCfin, add, dx, relu=True):
        C = fin.C
        coef = torch.empty(3 * C, dtype=fin.gamma.dtype, device=x.device)
        dg = fin.dgamma if fin.publish else torch.empty_like(fin.gamma)
        db = fin.dbeta if fin.publish else torch.empty_like(fin.gamma)
        self.bn_finalize_bwd(fin.stats, fin.G, fin.count, fin.gamma, fin.invstd, dg, db, coef)
        self.bn_bwd_apply(dy, dpool, pool_hw, x, scale, shift, fin.mean, fin.invstd, coef, add, dx, relu=relu)


class HipBackend(_Common):
    name = "hip"
    act_dtype = torch.bfloat16
    acc_dtype = torch.float32
    # replicas of every BN statistics accumulator: producer block b adds into replica b % R,
    # the finalize kernels sum them (same-address fp32 atomics serialize at ~15 ns each)
    stats_replicas = 8  # measured: 8 ~ 4 < 16 < 32 < 64

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.L = _lib.lib()
        # 4 KiB of device zeros: the padding source of the LDS-DMA conv loader
        self.zero_page = torch.zeros(1024, dtype=torch.float32, device=self.device)
        # conv kernel config per geometry key (set by the autotuner; -1 = library default)
        self.conv_cfg: dict = {}          # geometry key -> (config id, split-K factor)
        # split-K conv launches (DrnConvFwdArgs.ksplit): fp32 partial-tile workspace (grown before
        # any graph capture: the autotuner sizes it) and one ticket word per output tile
        self.ks_ws = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.ks_tickets = torch.zeros(1 << 16, dtype=torch.int32, device=self.device)
        self.KS_FACTORS = (2, 3, 4)
        # stream-K grid sizes tried by the autotuner (256 CUs: 1 or 2 resident workgroups each)
        self.SK_BLOCKS = (256, 512)
        # a fixed configuration for every conv (tests / experiments set it; None = autotune)
        self.forced_cfg = None
        self.autotune = os.environ.get("DRN_AUTOTUNE", "1") == "1"
        self.wgrad_ns: dict = {}
        # split-K by fp32 atomics into the gradient is a tuner candidate only once the executor
        # guarantees zeroed gradients at the start of every backward (wgrad_atomic_ok); it sets
        # wgrad_atomic_used when some layer picked it
        self.wgrad_atomic_ok = False
        self.wgrad_atomic_used = False
        self.forced_wgrad_ns = None  # a fixed weight-gradient pipeline (tests / experiments)
        self.tune_log: list = []
        self._db = None   # persistent kernel-selection database (ops/tunedb.py), loaded on first use
        self.db_hits = 0
        # tuner effort: first-pass launches per candidate, finalists re-timed, re-timing rounds
        # (scripts/make_tune_db.py raises them when it builds the shipped database)
        self.tune_iters = int(os.environ.get("DRN_TUNE_ITERS", "5"))
        self.tune_top = int(os.environ.get("DRN_TUNE_TOP", "4"))
        self.tune_rounds = int(os.environ.get("DRN_TUNE_ROUNDS", "2"))
        self._fin_bufs: dict = {}
        self.conv_cands: dict = {}   # geometry key -> tuner finalists, fastest first
        self._insitu = None          # list of (key, cfg, ev0, ev1) while Executor.insitu_tune runs
        self.recording = False       # a native step plan is being recorded (runtime/plan.py)

    def _timed(self, launch, n: int) -> float:
        """Mean ms of n back-to-back launches of launch() on the current stream."""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(n):
            launch()
        ev1.record()
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / n

    def tune_db(self):
        if self._db is None:
            from .tunedb import TuneDB, section_for
            self._db = TuneDB(section_for(self.device, self.L))
        return self._db

    def save_tune_db(self) -> bool:
        """Persist the configurations timed by this process (no-op when nothing new was tuned)."""
        return self._db is not None and self._db.save()

    def stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    # -- conv ---------------------------------------------------------------------------------
    def conv_args(self, x, w, y, g: ConvGeom, in_bn=None, relu_in=True, residual=None, stats=None, out_map=None,
                  bn_bwd=None, bn_fin: Optional[BnFin] = None, in_fin: Optional[BnCfin] = None):
        N, H, W, C = x.shape
        K, R, S, C2 = w.shape
        N2, P, Q, K2 = y.shape
        oH, oW = P, Q
        if out_map is not None:
            P, Q = out_map.P, out_map.Q
        assert C == C2 and K == K2 and N == N2, (x.shape, w.shape, y.shape)
        assert x.is_contiguous() and w.is_contiguous() and y.is_contiguous()
        a = _lib.DrnConvFwdArgs()
        a.x, a.w, a.y = x.data_ptr(), w.data_ptr(), y.data_ptr()
        a.in_scale = _ptr(in_bn[0]) if in_bn is not None else None
        a.in_shift = _ptr(in_bn[1]) if in_bn is not None else None
        a.residual = _ptr(residual)
        a.stats = _ptr(stats)
        a.N, a.H, a.W, a.C, a.K, a.R, a.S, a.P, a.Q = N, H, W, C, K, R, S, P, Q
        a.stride, a.pad_h, a.pad_w, a.dil = g.stride, g.pad_h, g.pad_w, g.dil
        a.fd_pq = _lib.DrnFastDiv.make(P * Q)
        a.fd_q = _lib.DrnFastDiv.make(Q)
        a.relu_in = 1 if relu_in else 0
        if out_map is not None:
            a.out_H, a.out_W, a.out_stride, a.out_oh, a.out_ow = oH, oW, out_map.stride, out_map.oh, out_map.ow
        if stats is not None:
            assert stats.numel() % (2 * K) == 0 and stats.dtype == torch.float32, \
                "stats accumulator must be fp32 [rep][2][K]"
            a.stats_rep = stats.numel() // (2 * K)
        if bn_bwd is not None:
            assert stats is not None, "fused BN-backward reduction accumulates into stats"
            bx, bsc, bsh, bmu, bis = bn_bwd
            assert bx.shape == y.shape
            a.bn_x, a.bn_scale, a.bn_shift = bx.data_ptr(), bsc.data_ptr(), bsh.data_ptr()
            a.bn_mean, a.bn_invstd = bmu.data_ptr(), bis.data_ptr()
        if bn_fin is not None:
            assert stats is not None and bn_fin.counters.dtype == torch.int32 and bn_fin.counters.numel() >= (K + 63) // 64
            f = bn_fin
            a.fin_cnt = f.counters.data_ptr()
            a.fin_count, a.fin_eps, a.fin_momentum = float(f.count), float(f.eps), float(f.momentum)
            a.fin_gamma = f.gamma.data_ptr()
            if bn_bwd is not None:
                a.fin_dgamma, a.fin_dbeta, a.fin_coef = f.dgamma.data_ptr(), f.dbeta.data_ptr(), f.coef.data_ptr()
            else:
                a.fin_beta = f.beta.data_ptr()
                a.fin_run_mean, a.fin_run_var = _ptr(f.run_mean), _ptr(f.run_var)
                a.fin_scale, a.fin_shift = f.scale.data_ptr(), f.shift.data_ptr()
                a.fin_mean, a.fin_invstd = f.mean.data_ptr(), f.invstd.data_ptr()
        if in_fin is not None:
            assert in_bn is not None and in_fin.C == C, "the consumer-side finalize feeds the fused BN prologue"
            _aligned16(in_fin.stats)
            a.in_fin = in_fin.struct()
        cfg, ks = (self.forced_cfg, 1) if self.forced_cfg is not None else self.conv_cfg.get(self.conv_key(a), (-1, 1))
        a.cfg = cfg
        self._set_ksplit(a, ks)
        # the struct holds raw device pointers: it keeps its tensors alive (a caller passing
        # temporaries, e.g. conv_args(x.cuda(), ...), must not launch on freed memory)
        a._keep = (x, w, y, in_bn, residual, stats, bn_bwd)
        return a

    def _ks_need(self, a, ks: int) -> int:
        """fp32 elements of split-K workspace a launch of config a.cfg with factor ks needs."""
        bp, bc = self.L.drn_conv_glds_cfg_bp(a.cfg), self.L.drn_conv_glds_cfg_bc(a.cfg)
        if bp <= 0 or bc <= 0:
            return 0
        M = a.N * a.P * a.Q
        return ((M + bp - 1) // bp) * ((a.K + bc - 1) // bc) * ks * bp * bc

    def _set_ksplit(self, a, ks: int):
        """ks > 1: split-K factor; ks < 0: stream-K over -ks workgroups (DrnConvFwdArgs.sk_blocks;
        ksplit then holds the partial slots per tile the launch needs)."""
        a.sk_blocks = 0
        a.ksplit = int(ks) if ks and ks > 1 else 0
        if ks and ks < 0:
            a.sk_blocks = -int(ks)
            a.ksplit = self.L.drn_conv_sk_slots_cfg(ctypes.byref(a), a.cfg, a.sk_blocks)
            if a.ksplit == 0:  # not applicable: leave it to the library to refuse the launch
                a.ks_ws = a.ks_tickets = None
                return
        if a.ksplit > 1 or a.sk_blocks:
            need = self._ks_need(a, max(1, a.ksplit))
            if need > self.ks_ws.numel():
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("split-K workspace must be sized before graph capture (autotune first)")
                # a recorded native plan / captured graph keeps the raw pointer of the old buffer:
                # it stays referenced (never freed under a live plan), the growth is monotone
                HipBackend._retired_ws.append(self.ks_ws)
                self.ks_ws = torch.empty(need, dtype=torch.float32, device=self.device)
            a.ks_ws, a.ks_tickets = self.ks_ws.data_ptr(), self.ks_tickets.data_ptr()

    @staticmethod
    def conv_key(a) -> tuple:
        """Geometry + every launch property a configuration's validity depends on (fused prologue
        with / without ReLU, consumer-side finalize replicas, strided output, epilogue operands)."""
        return (a.N, a.H, a.W, a.C, a.K, a.R, a.S, a.P, a.Q, a.stride, a.pad_h, a.pad_w, a.dil,
                a.in_scale is not None, a.out_stride, a.residual is not None, a.bn_x is not None,
                a.stats is not None, int(a.relu_in) if a.in_scale is not None else 0,
                int(a.in_fin.G) if a.in_fin.stats is not None else 0)

    def _conv_hit_ok(self, a, hit) -> bool:
        """A database choice is used only if this library can launch it for this geometry now
        (a known configuration, split-K / stream-K only on split-capable ones; the experiment
        candidate filter DRN_CONV_CANDS applies to hits too) -- otherwise the geometry is re-tuned."""
        cfg, ks = hit
        cands = os.environ.get("DRN_CONV_CANDS")
        if cands and cfg not in [int(c) for c in cands.split(",")]:
            return False
        nk0 = self.L.drn_conv_nk_cfg0()
        if cfg == 100:
            return ks == 1
        if nk0 <= cfg < nk0 + self.L.drn_conv_nk_num_cfgs():
            return ks == 1 and a.K in (16, 32)
        if not (0 <= cfg < self.L.drn_conv_glds_num_cfgs()) or not self.L.drn_conv_glds_ok(ctypes.byref(a)):
            return False
        if ks > 1:
            return self.L.drn_conv_glds_cfg_bk(cfg) > 0 and a.out_stride == 0
        if ks < 0:
            return a.out_stride == 0 and self.L.drn_conv_sk_slots_cfg(ctypes.byref(a), cfg, -ks) > 0
        return True

    def launch_conv(self, a):
        if a.cfg == -1 and self.autotune and self.forced_cfg is None:
            key = self.conv_key(a)
            if key not in self.conv_cfg and (self.recording or torch.cuda.is_current_stream_capturing()):
                raise RuntimeError(f"untuned convolution {key} while recording a step (tune it eagerly first)")
            if key not in self.conv_cfg:
                hit = self.tune_db().get_conv(key)
                if hit is not None and self._conv_hit_ok(a, hit):
                    self.db_hits += 1
                    self.conv_cfg[key] = hit
                else:
                    self.conv_cfg[key] = self._tune_conv(a, key)
                    self.tune_db().put_conv(key, self.conv_cfg[key])
            cfg, ks = self.conv_cfg.get(key, (-1, 1))
            a.cfg = cfg
            self._set_ksplit(a, ks)
        if self._insitu is not None:   # in-situ re-timing (Executor.insitu_tune): events around it
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.check(self.L.drn_conv_fwd2(ctypes.byref(a), self.zero_page.data_ptr(), self.stream()), "drn_conv_fwd")
            e1.record()
            self._insitu.append((self.conv_key(a), (int(a.cfg), self._ks_of(a)), e0, e1))
            return
        _lib.check(self.L.drn_conv_fwd2(ctypes.byref(a), self.zero_page.data_ptr(), self.stream()), "drn_conv_fwd")

    @staticmethod
    def _ks_of(a) -> int:
        """The split-K / stream-K factor a launch was configured with (inverse of _set_ksplit)."""
        return -int(a.sk_blocks) if a.sk_blocks else (int(a.ksplit) if a.ksplit > 1 else 1)

    def _tune_conv(self, a, key, iters: int = 0) -> int:
        """Time every kernel configuration for this geometry (the MIOpen 'find' step, done once
        per distinct convolution before the step is captured) and return the fastest. Runs on
        scratch outputs / statistics so no live buffer is modified. Every configuration
        accumulates each output in the same k order, so the choice does not change numerics."""
        if not self.L.drn_conv_glds_ok(ctypes.byref(a)):
            return (100, 1)
        iters = iters or self.tune_iters
        N, K = a.N, a.K
        oh = a.out_H if a.out_stride else a.P
        ow = a.out_W if a.out_stride else a.Q
        y = torch.empty(N * oh * ow * K, dtype=torch.bfloat16, device=self.device)
        st = torch.zeros(max(1, a.stats_rep) * 2 * K, dtype=torch.float32, device=self.device)  # all replicas
        t = _lib.DrnConvFwdArgs()
        ctypes.memmove(ctypes.addressof(t), ctypes.addressof(a), ctypes.sizeof(a))
        t.y = y.data_ptr()
        if a.residual is not None and a.residual == a.y:
            t.residual = t.y  # accumulating launch: time the same in-place epilogue on the scratch output
        if a.stats is not None:
            t.stats = st.data_ptr()
        t.fin_cnt = None  # timing runs must not finalize (moving averages) the live BN
        t.in_fin.publish = 0
        s = self.stream()
        cands = os.environ.get("DRN_CONV_CANDS")
        if cands:
            cands = [int(c) for c in cands.split(",")]
        else:  # register-staged, LDS-DMA and narrow-output (K = 16 / 32) configurations
            nk0 = self.L.drn_conv_nk_cfg0()
            cands = [100] + list(range(self.L.drn_conv_glds_num_cfgs())) + \
                [nk0 + i for i in range(self.L.drn_conv_nk_num_cfgs())] * (a.K in (16, 32))

        def setk(c):
            t.cfg, ks = c
            self._set_ksplit(t, ks)

        def time_cfg(c, n):
            setk(c)
            launch = lambda: _lib.check(self.L.drn_conv_fwd2(ctypes.byref(t), self.zero_page.data_ptr(), s),  # noqa
                                        "drn_conv_fwd")
            launch()
            return self._timed(launch, n)

        # candidates: (config, split-K factor); split-K only where the grid leaves CUs idle
        M = a.N * a.P * a.Q
        pairs = []
        for cfg in cands:
            pairs.append((cfg, 1))
            bp = self.L.drn_conv_glds_cfg_bp(cfg) if 0 <= cfg < 1000 else 0
            bc = self.L.drn_conv_glds_cfg_bc(cfg) if 0 <= cfg < 1000 else 0
            if bp > 0 and bc > 0 and a.out_stride == 0:
                tiles = ((M + bp - 1) // bp) * ((a.K + bc - 1) // bc)
                if tiles < 512:
                    pairs += [(cfg, k) for k in self.KS_FACTORS if k > 1]
                if tiles < 1024:  # stream-K: every CU gets the same share of tile k-stages
                    pairs += [(cfg, -g) for g in self.SK_BLOCKS if self.L.drn_conv_sk_slots_cfg(ctypes.byref(a), cfg, g)]
        # pass 1: every applicable configuration, short; pass 2: the 4 fastest re-timed twice,
        # interleaved, keeping each one's best (single short timings picked outliers: clock
        # ramps and neighbours' cache state moved the choice by >10 %)
        first = []
        for c in pairs:
            setk(c)
            if self.L.drn_conv_fwd2(ctypes.byref(t), self.zero_page.data_ptr(), s) != 0:
                continue  # configuration not applicable to this geometry (e.g. C % 64 != 0)
            first.append((time_cfg(c, iters), c))
        first.sort()
        top = {c: ms for ms, c in first[:self.tune_top]}
        for _ in range(self.tune_rounds if len(top) > 1 else 0):
            for c in list(top):
                top[c] = min(top[c], time_cfg(c, 2 * iters))
        best, best_t = min(top.items(), key=lambda kv: kv[1]) if top else ((100, 1), 0.0)
        self.tune_log.append((key, best, round(best_t * 1e3, 1)))
        # the finalists, fastest first: Executor.insitu_tune re-times them inside a real step
        self.conv_cands[key] = [c for c, _ in sorted(top.items(), key=lambda kv: kv[1])]
        return best

    def conv_fwd(self, x, w, y, g, in_bn=None, relu_in=True, residual=None, stats=None, out_map=None, bn_bwd=None,
                 bn_fin: Optional[BnFin] = None, out_fill: bool = False, in_fin: Optional[BnCfin] = None):
        """y = conv(x) (+ residual); optional BN statistics of y, or (bn_bwd = (x_bn, scale, shift,
        mean, invstd)) the fused BN-backward reduction with ReLU-masked output; bn_fin finalizes
        that BN in the same launch. out_fill (strided out_map, single-phase output): the epilogue
        also writes zeros at every other phase position, so y needs no separate clearing.
        in_fin: the input BN (in_bn) is finalized by this conv's prologue (BnCfin)."""
        a = self.conv_args(x, w, y, g, in_bn, relu_in, residual, stats, out_map, bn_bwd, bn_fin, in_fin)
        if out_fill:
            assert out_map is not None and bn_bwd is None and residual is None, "out_fill: plain strided output only"
            a.out_fill = 1
        self.launch_conv(a)

    WGRAD_TARGET_BLOCKS = 512  # measured: 512 > 384, 640, 1024
    WGRAD_MIN_STEPS = 8

    @staticmethod
    def wgrad_splits(M, Ktot, K, target_blocks: int = 0, min_steps: int = 0):
        """Split-K over output pixels: enough workgroups to fill 256 CUs (~2.5 per CU) while
        keeping >= min_steps 64-pixel steps per split so partial slabs stay cheap."""
        target_blocks = target_blocks or HipBackend.WGRAD_TARGET_BLOCKS
        min_steps = min_steps or HipBackend.WGRAD_MIN_STEPS
        bkk = 128 if Ktot > 64 else 64
        bco = 128 if K > 64 else 64
        if K <= 32:  # the narrow-output tiles of csrc/kernels/conv_wgrad.hip dispatch_wgrad_tile
            bco = 32
            bkk = 128 if (Ktot > 64 and -(-Ktot // 128) * 128 <= -(-Ktot // 64) * 64) else 64
        tiles = ((Ktot + bkk - 1) // bkk) * ((K + bco - 1) // bco)
        steps = (M + 63) // 64
        # never MORE blocks than the target (rounding the split count up made e.g. 36 tiles x 15
        # splits = 540 blocks for a 512-slot target: 28 blocks ran as a second wave, alone)
        want = max(1, min(target_blocks // tiles, max(1, steps // min_steps)))
        per = (steps + want - 1) // want
        splits = (steps + per - 1) // per
        return splits, per * 64

    # split-K block targets the wgrad autotuner chooses from per geometry: more splits fill the
    # chip, fewer write (and re-read in drn_splitk_reduce) fewer fp32 partial slabs -- the slab
    # traffic of the default 512-block target is ~1.7 GB per ResNet-50 step
    WGRAD_TARGETS = (128, 256, 384, 512, 768)
    # minimum 64-pixel steps per split the tuner also tries: small layers (CIFAR stage 3 at batch
    # 32: 32 steps) otherwise get 4 splits, i.e. 20-64 workgroups walking 8 serial steps each
    WGRAD_MIN_STEPS_CANDS = (8, 2)

    def wgrad_args(self, x, dy, out, g: ConvGeom, in_bn=None, relu_in=True, ws=None, target_blocks: int = 0,
                   atomic: bool = False, min_steps: int = 0):
        N, H, W, C = x.shape
        N2, P, Q, K = dy.shape
        Kd, R, S, Cd = out.shape
        assert Kd == K and Cd == C and N == N2
        M = N * P * Q
        splits, pps = self.wgrad_splits(M, R * S * C, K, target_blocks, min_steps)
        a = _lib.DrnConvWgradArgs()
        a.x, a.dy = x.data_ptr(), dy.data_ptr()
        a.in_scale = _ptr(in_bn[0]) if in_bn is not None else None
        a.in_shift = _ptr(in_bn[1]) if in_bn is not None else None
        a.N, a.H, a.W, a.C, a.K, a.R, a.S, a.P, a.Q = N, H, W, C, K, R, S, P, Q
        a.stride, a.pad_h, a.pad_w = g.stride, g.pad_h, g.pad_w
        a.relu_in = 1 if relu_in else 0
        a.splits, a.pix_per_split = splits, pps
        a.fd_pq = _lib.DrnFastDiv.make(P * Q)
        a.fd_q = _lib.DrnFastDiv.make(Q)
        if splits == 1 or atomic:
            a.out = out.data_ptr()
            a.atomic_out = 1 if (atomic and splits > 1) else 0
        else:
            need = splits * out.numel()
            assert ws is not None and ws.numel() >= need, f"wgrad workspace too small ({need})"
            a.out = ws.data_ptr()
        a._keep = (x, dy, out, in_bn, ws)  # (raw pointers above: keep the tensors alive)
        return a

    def wgrad_ws_elems(self, M, K, R, S, C):
        """Workspace for the largest split count any candidate target can choose."""
        need = 0
        for t in set(self.WGRAD_TARGETS) | {self.WGRAD_TARGET_BLOCKS}:
            for ms in set(self.WGRAD_MIN_STEPS_CANDS) | {self.WGRAD_MIN_STEPS}:
                splits, _ = self.wgrad_splits(M, R * S * C, K, t, ms)
                if splits > 1:
                    need = max(need, splits * K * R * S * C)
        return need

    @staticmethod
    def wgrad_key(a) -> tuple:
        return (a.N, a.H, a.W, a.C, a.K, a.R, a.S, a.P, a.Q, a.stride, a.pad_h, a.pad_w, a.in_scale is not None)

    def _wgrad_kernel(self, a, ns: int, st):
        _lib.check(self.L.drn_conv_wgrad2(ctypes.byref(a), self.zero_page.data_ptr(), ns, st), "drn_conv_wgrad")

    def _wgrad_full(self, a, ns: int, out, st):
        self._wgrad_kernel(a, ns, st)
        if a.splits > 1 and not a.atomic_out:
            _lib.check(self.L.drn_splitk_reduce(a.out, out.data_ptr(), out.numel(), a.splits, 1.0, 0, st),
                       "drn_splitk_reduce")

    def _tune_wgrad(self, args_for, out, key, iters: int = 0) -> tuple:
        """Pick (split-K target, pipeline) by timing the weight-gradient kernel TOGETHER with its
        split-K reduction: 0 = register-staged, 2/3 = LDS-DMA stages of 64 pixels, 4/5/6 = 2/3/4
        stages of 32 pixels, 7/8 = the interleaved-issue 64-pixel pipelines, 9/10 = the packed
        stem's input-halo kernel with 3/4 stages (other geometries refuse it). Writes only the workspace and this gradient slot (rewritten by the
        real launch that follows)."""
        iters = iters or self.tune_iters
        st = self.stream()
        cands = tuple(int(c) for c in os.environ.get("DRN_WGRAD_CANDS", "0,2,3,4,5,6,7,8,9,10").split(","))
        seen = set()
        modes = (False, True) if self.wgrad_atomic_ok else (False,)

        def time_one(a, ns, n):
            return self._timed(lambda: self._wgrad_full(a, ns, out, st), n)

        first = []  # (ms, (target, pipeline, atomic, min steps), args)
        for tgt, atomic, ms_min in [(t, m, k) for t in self.WGRAD_TARGETS for m in modes
                                    for k in self.WGRAD_MIN_STEPS_CANDS]:
            a = args_for(tgt, atomic, ms_min)
            if (a.splits, a.atomic_out) in seen:
                continue
            seen.add((a.splits, a.atomic_out))
            for ns in cands:
                if self.L.drn_conv_wgrad2(ctypes.byref(a), self.zero_page.data_ptr(), ns, st) != 0:
                    continue  # pipeline not available for this launch
                for _ in range(2):
                    self._wgrad_full(a, ns, out, st)
                first.append((time_one(a, ns, iters), (tgt, ns, bool(a.atomic_out), ms_min), a))
        if not first:
            return (0, 2, False, 0)
        # pass 2 (as the forward tuner): the 4 fastest re-timed twice, interleaved, each keeping its
        # best -- single 5-launch timings of ~10-us CIFAR kernels picked outliers (run-to-run step
        # spread 1.77-1.95 ms at batch 32)
        first.sort(key=lambda r: r[0])
        top = [[ms, cfg, a] for ms, cfg, a in first[:self.tune_top]]
        for _ in range(self.tune_rounds if len(top) > 1 else 0):
            for r in top:
                r[0] = min(r[0], time_one(r[2], r[1][1], 2 * iters))
        best_t, best, _ = min(top, key=lambda r: r[0])
        if best[2]:
            self.wgrad_atomic_used = True  # the executor now zeroes the gradients every step
        self.tune_log.append((("wgrad",) + key, best, round(best_t * 1e3, 1)))
        return best

    def conv_wgrad(self, x, dy, out, g, in_bn=None, relu_in=True, ws=None):
        args_for = lambda tgt, atomic=False, ms=0: self.wgrad_args(x, dy, out, g, in_bn, relu_in, ws, tgt, atomic, ms)
        a = args_for(0)
        st = self.stream()
        if self.forced_wgrad_ns is not None:
            self._wgrad_full(a, self.forced_wgrad_ns, out, st)
            return
        key = self.wgrad_key(a)
        if key not in self.wgrad_ns and self.autotune and self.recording:
            raise RuntimeError(f"untuned weight gradient {key} while recording a step (tune it eagerly first)")
        if key not in self.wgrad_ns and self.autotune and not torch.cuda.is_current_stream_capturing():
            hit = self.tune_db().get_wgrad(key)
            cands = [int(c) for c in os.environ.get("DRN_WGRAD_CANDS", "0,2,3,4,5,6,7,8,9,10").split(",")]
            if hit is not None and (not hit[2] or self.wgrad_atomic_ok) and hit[1] in cands:
                self.db_hits += 1
                self.wgrad_ns[key] = hit
                if hit[2]:
                    self.wgrad_atomic_used = True  # the executor now zeroes the gradients every step
            else:
                self.wgrad_ns[key] = self._tune_wgrad(args_for, out, key)
                self.tune_db().put_wgrad(key, self.wgrad_ns[key])
            if self.wgrad_ns[key][2]:
                self.zero_(out)  # the timing launches left partial sums in this gradient slot
        tgt, ns, atomic, ms = self.wgrad_ns.get(key, (0, 2, False, 0))
        if tgt or atomic or ms:
            a = args_for(tgt, atomic, ms)
        self._wgrad_full(a, ns, out, st)

    # -- batch norm -----------------------------------------------------------------------------
    @staticmethod
    def bn_rows_per_block(M, C):
        rpp = max(1, 256 // (C // 8))
        G_target = 512
        rpb = max(rpp, ((M + G_target - 1) // G_target + rpp - 1) // rpp * rpp)
        return rpb

    def bn_stats(self, x, part):
        """part[R][2][C] += (sum, sumsq) over rows of x (block b into replica b % R); returns R."""
        C = x.shape[-1]
        M = x.numel() // C
        rpb = self.bn_rows_per_block(M, C)
        _lib.check(self.L.drn_bn_stats(x.data_ptr(), part.data_ptr(), M, C, rpb, part.numel() // (2 * C),
                                       self.stream()), "drn_bn_stats")
        return part.numel() // (2 * C)

    def bn_finalize(self, part, G, count, gamma, beta, run_mean, run_var, scale, shift, mean, invstd,
                    momentum, eps, update_running=True):
        C = gamma.numel()
        _lib.check(self.L.drn_bn_finalize(part.data_ptr(), G, C, float(count), gamma.data_ptr(), beta.data_ptr(),
                                          eps, momentum, _ptr(run_mean) if update_running else None,
                                          _ptr(run_var) if update_running else None, scale.data_ptr(),
                                          shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(), self.stream()),
                   "drn_bn_finalize")

    def bn_inference(self, gamma, beta, run_mean, run_var, eps, scale, shift, mean=None, invstd=None):
        _lib.check(self.L.drn_bn_inference_params(gamma.numel(), gamma.data_ptr(), beta.data_ptr(),
                                                  run_mean.data_ptr(), run_var.data_ptr(), eps, scale.data_ptr(),
                                                  shift.data_ptr(), _ptr(mean), _ptr(invstd), self.stream()),
                   "drn_bn_inference_params")

    def bn_apply(self, x, y, scale, shift, relu=True):
        C = x.shape[-1]
        _lib.check(self.L.drn_bn_apply(x.data_ptr(), y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                       x.numel() // C, C, 1 if relu else 0, self.stream()), "drn_bn_apply")

    def bn_apply_stats(self, x, y, acc, count, gamma, beta, run_mean, run_var, scale, shift, mean, invstd,
                       momentum, eps, relu=True):
        C = x.shape[-1]
        _aligned16(acc, gamma, beta, run_mean, run_var, scale, shift, mean, invstd)
        _lib.check(self.L.drn_bn_apply_stats(x.data_ptr(), y.data_ptr(), acc.data_ptr(), float(count),
                                             gamma.data_ptr(), beta.data_ptr(), float(eps), float(momentum),
                                             run_mean.data_ptr(), run_var.data_ptr(), scale.data_ptr(),
                                             shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(), x.numel() // C, C,
                                             1 if relu else 0, self.stream()), "drn_bn_apply_stats")

    def bn_bwd_apply_stats(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, acc, count, gamma, dgamma,
                           dbeta, add, dx, coef=None, relu=True):
        C = x.shape[-1]
        _aligned16(acc, gamma, dgamma, dbeta, scale, shift, mean, invstd)
        _lib.check(self.L.drn_bn_bwd_apply_stats(_ptr(dy), _ptr(dpool), pool_hw, x.data_ptr(), scale.data_ptr(),
                                                 shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                                 acc.data_ptr(), float(count), gamma.data_ptr(), dgamma.data_ptr(),
                                                 dbeta.data_ptr(), _ptr(add), dx.data_ptr(), x.numel() // C, C,
                                                 1 if relu else 0, self.stream()), "drn_bn_bwd_apply_stats")

    def bn_apply_fin(self, x, y, fin: BnCfin, relu=True):
        C = x.shape[-1]
        if C >= self.BN_FIN_SPLIT_C and fin.publish:
            # (the publishing consumer: one finalize launch writes scale / shift / moving
            # averages, the plain apply reads them; a non-publishing consumer keeps the fused
            # prologue, since nothing orders it after the publisher)
            self.bn_finalize(fin.stats, fin.G, fin.count, fin.gamma, fin.beta, fin.run_mean, fin.run_var, fin.scale,
                             fin.shift, fin.mean, fin.invstd, fin.momentum, fin.eps,
                             update_running=fin.run_mean is not None)
            self.bn_apply(x, y, fin.scale, fin.shift, relu=relu)
            return
        f = fin.struct()
        _lib.check(self.L.drn_bn_apply_fin(x.data_ptr(), y.data_ptr(), ctypes.byref(f), x.numel() // C, C,
                                           1 if relu else 0, self.stream()), "drn_bn_apply_fin")

    # consumer-side finalize costs every workgroup of the apply C channels x G replicas of L2
    # reads in its prologue (2048 workgroups x 2048 channels x 64 B = 268 MB at the last stage of
    # ResNet-50): from this many channels on, one small finalize launch computes the
    # coefficients once and the apply reads only its own 8 channels'
    BN_FIN_SPLIT_C = 1024

    def _fin_scratch(self, C: int) -> torch.Tensor:
        """[coef 3C][dgamma C][dbeta C] fp32 scratch of the split backward finalize (one per C:
        the BatchNorm-backward applies run in order on one stream); allocated by the eager
        warm-up step, before any graph capture."""
        buf = self._fin_bufs.get(C)
        if buf is None:
            buf = self._fin_bufs[C] = torch.empty(5 * C, dtype=torch.float32, device=self.device)
        return buf

    def bn_bwd_apply_fin(self, dy, dpool, pool_hw, x, scale, shift, fin: BnCfin, add, dx, relu=True):
        C = x.shape[-1]
        _aligned16(scale, shift)
        if C >= self.BN_FIN_SPLIT_C:
            buf = self._fin_scratch(C)
            coef = buf[:3 * C]
            dg = fin.dgamma if fin.publish else buf[3 * C:4 * C]
            db = fin.dbeta if fin.publish else buf[4 * C:]
            self.bn_finalize_bwd(fin.stats, fin.G, fin.count, fin.gamma, fin.invstd, dg, db, coef)
            self.bn_bwd_apply(dy, dpool, pool_hw, x, scale, shift, fin.mean, fin.invstd, coef, add, dx, relu=relu)
            return
        f = fin.struct()
        _lib.check(self.L.drn_bn_bwd_apply_fin(_ptr(dy), _ptr(dpool), pool_hw, x.data_ptr(), scale.data_ptr(),
                                               shift.data_ptr(), ctypes.byref(f), _ptr(add), dx.data_ptr(),
                                               x.numel() // C, C, 1 if relu else 0, self.stream()),
                   "drn_bn_bwd_apply_fin")

    def bn_bwd_reduce(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, part, relu=True):
        C = x.shape[-1]
        M = x.numel() // C
        rpb = self.bn_rows_per_block(M, C)
        _lib.check(self.L.drn_bn_bwd_reduce(_ptr(dy), _ptr(dpool), pool_hw, x.data_ptr(), scale.data_ptr(),
                                            shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(),
                                            M, C, rpb, 1 if relu else 0, part.numel() // (2 * C), self.stream()),
                   "drn_bn_bwd_reduce")
        return part.numel() // (2 * C)

    def bn_finalize_bwd(self, part, G, count, gamma, invstd, dgamma, dbeta, coef):
        _lib.check(self.L.drn_bn_finalize_bwd(part.data_ptr(), G, gamma.numel(), float(count), gamma.data_ptr(),
                                              invstd.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(),
                                              coef.data_ptr(), self.stream()), "drn_bn_finalize_bwd")

    def bn_bwd_apply(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, coef, add, dx, relu=True):
        C = x.shape[-1]
        _lib.check(self.L.drn_bn_bwd_apply(_ptr(dy), _ptr(dpool), pool_hw, x.data_ptr(), scale.data_ptr(),
                                           shift.data_ptr(), mean.data_ptr(), invstd.data_ptr(), coef.data_ptr(),
                                           _ptr(add), dx.data_ptr(), x.numel() // C, C, 1 if relu else 0,
                                           self.stream()), "drn_bn_bwd_apply")

    # -- head -----------------------------------------------------------------------------------
    def pool_bnrelu(self, x, scale, shift, pooled, relu=True):
        N, H, W, C = x.shape
        _lib.check(self.L.drn_bnrelu_pool(x.data_ptr(), _ptr(scale), _ptr(shift), pooled.data_ptr(), N, H * W, C,
                                          1 if relu else 0, self.stream()), "drn_bnrelu_pool")

    _sgemm_ws: dict = {}
    # superseded split-K / sgemm workspaces: native step plans and HIP graphs replay raw device
    # pointers, so a workspace a plan may have recorded is never returned to the allocator
    # (growth is monotone, so this at most doubles the workspace footprint)
    _retired_ws: list = []
    SGEMM_TARGET_WG = 256

    def sgemm(self, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias=None):
        tiles = ((M + 63) // 64) * ((N + 63) // 64)
        splits = max(1, min(K // 128, self.SGEMM_TARGET_WG // max(tiles, 1)))  # fill the CUs on long-K GEMMs
        ws = None
        if splits > 1:
            # split-K partials: one workspace per stream (GEMMs on the weight-gradient side
            # stream run concurrently with the main stream's)
            need = splits * M * ldc
            key = (C.device, self.stream())
            ws = HipBackend._sgemm_ws.get(key)
            if ws is None or ws.numel() < need:
                if ws is not None:
                    if torch.cuda.is_current_stream_capturing():
                        raise RuntimeError("sgemm workspace must be sized before graph capture")
                    HipBackend._retired_ws.append(ws)  # (plans recorded earlier keep its pointer)
                ws = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=C.device)
                HipBackend._sgemm_ws[key] = ws
        _lib.check(self.L.drn_sgemm(int(ta), int(tb), M, N, K, float(alpha), A.data_ptr(), lda, B.data_ptr(), ldb,
                                    float(beta), C.data_ptr(), ldc, _ptr(bias), splits, _ptr(ws), self.stream()),
                   "drn_sgemm")

    def softmax_xent(self, logits, labels, grad_scale, dlogits, loss, correct, probs=None):
        N, ncls = logits.shape
        _lib.check(self.L.drn_softmax_xent(logits.data_ptr(), labels.data_ptr(), N, ncls, float(grad_scale),
                                           _ptr(dlogits), loss.data_ptr(), _ptr(probs), _ptr(correct),
                                           self.stream()), "drn_softmax_xent")

    def colsum(self, x, out, scale=1.0, accumulate=False):
        rows, cols = x.shape
        _lib.check(self.L.drn_colsum(x.data_ptr(), rows, cols, out.data_ptr(), float(scale), int(accumulate),
                                     self.stream()), "drn_colsum")

    # -- pooling --------------------------------------------------------------------------------
    def maxpool_fwd(self, x, y, arg, k, stride, pad_h, pad_w, stats=None):
        """stats (optional [R][2][C] fp32): += per-channel (sum, sumsq) of y, fused in the kernel."""
        N, H, W, C = x.shape
        _, P, Q, _ = y.shape
        rep = stats.numel() // (2 * C) if stats is not None else 0
        _lib.check(self.L.drn_maxpool_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), N, H, W, C, P, Q, k, stride,
                                          pad_h, pad_w, _ptr(stats), rep, self.stream()), "drn_maxpool_fwd")

    def maxpool_bwd(self, dy, arg, dx, k, stride, pad_h, pad_w):
        N, H, W, C = dx.shape
        _, P, Q, _ = dy.shape
        _lib.check(self.L.drn_maxpool_bwd(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, C, P, Q, k, stride,
                                          pad_h, pad_w, self.stream()), "drn_maxpool_bwd")

    # -- optimizer / weights ------------------------------------------------------------------------
    def sgd_momentum(self, w, m, g, wb, lr_t, momentum, wd, grad_scale, skip=None):
        """Fused SGD-momentum; skip = optional device int32 word: the launch changes nothing when
        it holds a non-zero value at run time (a failed P2P gradient exchange)."""
        assert g.dtype in (torch.float32, torch.bfloat16) and g.numel() == w.numel()
        _lib.check(self.L.drn_sgd_momentum(w.data_ptr(), m.data_ptr(), g.data_ptr(), int(g.dtype == torch.bfloat16),
                                           _ptr(wb), w.numel(), lr_t.data_ptr(), float(momentum), float(wd),
                                           float(grad_scale), _ptr(skip), self.stream()), "drn_sgd_momentum")

    def cast_bf16(self, x, y):
        _lib.check(self.L.drn_cast_bf16(x.data_ptr(), y.data_ptr(), x.numel(), self.stream()), "drn_cast_bf16")

    # -- packed stem (csrc/kernels/stem.hip) ---------------------------------------------------------
    def stem_pack_input(self, x, xp):
        """x [N,H,W,8] bf16 -> xp [N,H,W+2,4] (pad columns zeroed once by the caller)."""
        N, H, W, C = x.shape
        assert C == 8 and tuple(xp.shape) == (N, H, W + 2, 4) and xp.is_contiguous() and x.is_contiguous()
        _lib.check(self.L.drn_stem_pack_input(x.data_ptr(), xp.data_ptr(), N * H, W, self.stream()),
                   "drn_stem_pack_input")

    def stem_pack_weights(self, w, wp):
        K, R, S, C = w.shape
        K2, R2, S8, C4 = wp.shape
        assert (K2, R2) == (K, R) and w.dtype == wp.dtype == torch.bfloat16
        _lib.check(self.L.drn_stem_pack_weights(w.data_ptr(), wp.data_ptr(), K, R, S, C, S8, C4, self.stream()),
                   "drn_stem_pack_weights")

    def stem_conv_pool(self, xp, w4, y, arg, g, H, W, P, Q, stats=None):
        """Fused packed stem conv (xp [N,H,W+2,4], w4 [K,7,8,4], geometry g of the packed conv)
        + 3x3/2 max-pool into y / arg [N,ceil(P/2),ceil(Q/2),K]; stats (optional [R][2][K] fp32):
        += per-channel (sum, sumsq) of y (csrc/kernels/stem_pool.hip stem_conv_pool_kernel)."""
        N, PP, QP, K = y.shape
        assert tuple(xp.shape) == (N, H, W + 2, 4) and tuple(w4.shape) == (K, 7, 8, 4) and g.stride == 2
        assert arg.shape == y.shape and xp.is_contiguous() and w4.is_contiguous() and y.is_contiguous()
        rep = stats.numel() // (2 * K) if stats is not None else 0
        _lib.check(self.L.drn_stem_conv_pool(xp.data_ptr(), w4.data_ptr(), y.data_ptr(), arg.data_ptr(), _ptr(stats),
                                             rep, N, H, W, P, Q, PP, QP, K, g.pad_h, g.pad_w, self.stream()),
                   "drn_stem_conv_pool")

    def stem_unpack_grad(self, dwp, dw):
        K, R, S, C = dw.shape
        K2, R2, S8, C4 = dwp.shape
        assert (K2, R2) == (K, R) and dw.dtype == dwp.dtype == torch.float32 and dw.is_contiguous()
        _lib.check(self.L.drn_stem_unpack_grad(dwp.data_ptr(), dw.data_ptr(), K, R, S, C, S8, C4, self.stream()),
                   "drn_stem_unpack_grad")

    def weight_tflip(self, wb, wt, table, ntab, total):
        _lib.check(self.L.drn_weight_tflip(wb.data_ptr(), wt.data_ptr(), table.data_ptr(), ntab, total,
                                           self.stream()), "drn_weight_tflip")

    def zero_(self, t):
        """In-tree fill kernel (no PyTorch kernel in the step): fp32 buffers, or any contiguous
        buffer whose byte size is a multiple of 4 (zero bits are zero in every dtype)."""
        nb = t.numel() * t.element_size()
        if t.is_contiguous() and nb % 4 == 0 and t.data_ptr() % 4 == 0:
            _lib.check(self.L.drn_fill_f32(t.data_ptr(), nb // 4, 0.0, self.stream()), "drn_fill_f32")
        else:
            t.zero_()

    def fill_(self, t, v: float):
        assert t.dtype == torch.float32 and t.is_contiguous()
        _lib.check(self.L.drn_fill_f32(t.data_ptr(), t.numel(), float(v), self.stream()), "drn_fill_f32")

    # -- input ----------------------------------------------------------------------------------
    def cifar_augment(self, raw_u8, params_i32, out, pad):
        N, H, W, _ = raw_u8.shape
        _lib.check(self.L.drn_cifar_augment(raw_u8.data_ptr(), params_i32.data_ptr(), out.data_ptr(), N, H, W, pad,
                                            self.stream()), "drn_cifar_augment")

    def vgg_preprocess(self, packed_u8, desc_i32, out, means):
        N, OH, OW, _ = out.shape
        _lib.check(self.L.drn_vgg_preprocess(packed_u8.data_ptr(), desc_i32.data_ptr(), out.data_ptr(), N, OH, OW,
                                             float(means[0]), float(means[1]), float(means[2]), self.stream()),
                   "drn_vgg_preprocess")

    def synthetic_images(self, out, seed):
        N, H, W, C = out.shape
        assert C == 8
        _lib.check(self.L.drn_synthetic_images(out.data_ptr(), N * H * W, seed & 0xFFFFFFFF, self.stream()),
                   "drn_synthetic_images")


# ----------------------------------------------------------------------------------------------
# fp32 reference backend (CPU runs + test oracle)
# ----------------------------------------------------------------------------------------------
_DT = [torch.float32]  # compute dtype of the reference backend (float64 for exactness tests)


def _pre(x, in_bn, relu_in):
    if in_bn is None:
        return x.to(_DT[0])
    y = x.to(_DT[0]) * in_bn[0].to(_DT[0]) + in_bn[1].to(_DT[0])
    return torch.relu(y) if relu_in else y


def _pad_for(xc, P, Q, R, S, g: ConvGeom):
    """Pad/crop an NCHW (virtual) input so a VALID conv with stride g.stride yields P x Q."""
    Hv, Wv = xc.shape[2], xc.shape[3]
    pb = (P - 1) * g.stride + R - g.pad_h - Hv
    pr = (Q - 1) * g.stride + S - g.pad_w - Wv
    return F.pad(xc, (g.pad_w, pr, g.pad_h, pb))


def _dilate(xc, dil):
    if dil == 1:
        return xc
    N, C, H, W = xc.shape
    out = xc.new_zeros(N, C, (H - 1) * dil + 1, (W - 1) * dil + 1)
    out[:, :, ::dil, ::dil] = xc
    return out


class RefBackend(_Common):
    name = "ref"
    stats_replicas = 1

    def __init__(self, device="cpu", dtype=torch.float32):
        self.device = torch.device(device)
        self.act_dtype = dtype
        self.acc_dtype = dtype
        _DT[0] = dtype

    def stream(self):
        return None

    def conv_fwd(self, x, w, y, g: ConvGeom, in_bn=None, relu_in=True, residual=None, stats=None, out_map=None,
                 bn_bwd=None, bn_fin: Optional[BnFin] = None, out_fill: bool = False, in_fin: Optional[BnCfin] = None):
        if in_fin is not None and in_fin.publish:
            self._publish_fwd(in_fin)
        self._conv_fwd(x, w, y, g, in_bn, relu_in, residual, stats, out_map, bn_bwd, out_fill)
        if bn_fin is not None:
            f, G = bn_fin, stats.numel() // (2 * w.shape[0])
            if bn_bwd is not None:
                self.bn_finalize_bwd(stats, G, f.count, f.gamma, bn_bwd[4], f.dgamma, f.dbeta, f.coef)
            else:
                self.bn_finalize(stats, G, f.count, f.gamma, f.beta, f.run_mean, f.run_var, f.scale, f.shift, f.mean,
                                 f.invstd, f.momentum, f.eps, update_running=f.run_mean is not None)

    def _conv_fwd(self, x, w, y, g: ConvGeom, in_bn=None, relu_in=True, residual=None, stats=None, out_map=None,
                  bn_bwd=None, out_fill=False):
        K, R, S, C = w.shape
        _, P, Q, _ = y.shape
        if out_map is not None:
            P, Q = out_map.P, out_map.Q
        xc = _dilate(_pre(x, in_bn, relu_in).permute(0, 3, 1, 2), g.dil)
        xc = _pad_for(xc, P, Q, R, S, g)
        out = F.conv2d(xc, w.to(_DT[0]).permute(0, 3, 1, 2), stride=g.stride).permute(0, 2, 3, 1)
        sl = None
        if out_map is not None:
            sl = (slice(None), slice(out_map.oh, out_map.oh + (P - 1) * out_map.stride + 1, out_map.stride),
                  slice(out_map.ow, out_map.ow + (Q - 1) * out_map.stride + 1, out_map.stride))
            if residual is not None:
                out = out + residual[sl].to(_DT[0])
        elif residual is not None:
            out = out + residual.to(_DT[0])
        if bn_bwd is not None:
            bx, bsc, bsh, bmu, bis = bn_bwd
            xb = (bx[sl] if sl is not None else bx).to(_DT[0])
            out = out.to(y.dtype).to(_DT[0]) * ((xb * bsc + bsh) > 0).to(_DT[0])
            gg, xh = out.reshape(-1, K), ((xb - bmu) * bis).reshape(-1, K)
            stats.view(-1)[:K].add_(gg.sum(0))
            stats.view(-1)[K:2 * K].add_((gg * xh).sum(0))
        if sl is not None:
            if out_fill:
                y.zero_()
            y[sl] = out.to(y.dtype)
            return
        y.copy_(out)
        if stats is not None and bn_bwd is None:
            yy = y.to(_DT[0]).reshape(-1, K)
            stats.view(-1)[:K].add_(yy.sum(0))
            stats.view(-1)[K:2 * K].add_((yy * yy).sum(0))

    def wgrad_ws_elems(self, M, K, R, S, C):
        return 0

    def conv_wgrad(self, x, dy, out, g: ConvGeom, in_bn=None, relu_in=True, ws=None):
        K, R, S, C = out.shape
        _, P, Q, _ = dy.shape
        xc = _pad_for(_pre(x, in_bn, relu_in).permute(0, 3, 1, 2), P, Q, R, S, g)
        dw = torch.nn.grad.conv2d_weight(xc, (K, C, R, S), dy.to(_DT[0]).permute(0, 3, 1, 2), stride=g.stride)
        out.copy_(dw.permute(0, 2, 3, 1))

    def bn_stats(self, x, part):
        C = x.shape[-1]
        xx = x.to(_DT[0]).reshape(-1, C)
        part.view(-1)[:C].add_(xx.sum(0))
        part.view(-1)[C:2 * C].add_((xx * xx).sum(0))
        return 1

    def bn_finalize(self, part, G, count, gamma, beta, run_mean, run_var, scale, shift, mean, invstd,
                    momentum, eps, update_running=True):
        C = gamma.numel()
        p = part.view(-1)[:2 * C].view(2, C).double().clone()
        part.view(-1)[:2 * C].zero_()
        mu = p[0] / count
        var = (p[1] / count - mu * mu).clamp_min(0)
        istd = 1.0 / torch.sqrt(var + eps)
        scale.copy_(gamma * istd.to(_DT[0]))
        shift.copy_(beta - mu.to(_DT[0]) * scale)
        mean.copy_(mu.to(_DT[0]))
        invstd.copy_(istd.to(_DT[0]))
        if update_running:
            unb = var * count / (count - 1) if count > 1 else var
            run_mean.mul_(momentum).add_((1 - momentum) * mu.to(_DT[0]))
            run_var.mul_(momentum).add_((1 - momentum) * unb.to(_DT[0]))

    def bn_inference(self, gamma, beta, run_mean, run_var, eps, scale, shift, mean=None, invstd=None):
        istd = torch.rsqrt(run_var + eps)
        scale.copy_(gamma * istd)
        shift.copy_(beta - run_mean * scale)
        if mean is not None:
            mean.copy_(run_mean)
        if invstd is not None:
            invstd.copy_(istd)

    def bn_apply(self, x, y, scale, shift, relu=True):
        v = x.to(_DT[0]) * scale + shift
        y.copy_(torch.relu(v) if relu else v)

    def _dy(self, dy, dpool, pool_hw, x):
        if pool_hw > 0:
            N, H, W, C = x.shape
            return (dpool.view(N, 1, 1, C) / pool_hw).expand(N, H, W, C)
        return dy.to(_DT[0])

    def bn_bwd_reduce(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, part, relu=True):
        C = x.shape[-1]
        d = self._dy(dy, dpool, pool_hw, x).reshape(-1, C)
        xx = x.to(_DT[0]).reshape(-1, C)
        if relu:
            d = d * ((xx * scale + shift) > 0).to(_DT[0])
        xh = (xx - mean) * invstd
        part.view(-1)[:C].add_(d.sum(0))
        part.view(-1)[C:2 * C].add_((d * xh).sum(0))
        return 1

    def bn_finalize_bwd(self, part, G, count, gamma, invstd, dgamma, dbeta, coef):
        C = gamma.numel()
        p = part.view(-1)[:2 * C].view(2, C).double().clone()
        part.view(-1)[:2 * C].zero_()
        dbeta.copy_(p[0].to(_DT[0]))
        dgamma.copy_(p[1].to(_DT[0]))
        coef.view(3, C)[0].copy_(gamma * invstd)
        coef.view(3, C)[1].copy_((p[0] / count).to(_DT[0]))
        coef.view(3, C)[2].copy_((p[1] / count).to(_DT[0]))

    def bn_bwd_apply(self, dy, dpool, pool_hw, x, scale, shift, mean, invstd, coef, add, dx, relu=True):
        C = x.shape[-1]
        shp = x.shape
        d = self._dy(dy, dpool, pool_hw, x).reshape(-1, C)
        xx = x.to(_DT[0]).reshape(-1, C)
        if relu:
            d = d * ((xx * scale + shift) > 0).to(_DT[0])
        xh = (xx - mean) * invstd
        k = coef.view(3, C)
        v = k[0] * (d - k[1] - xh * k[2])
        if add is not None:
            v = v + add.to(_DT[0]).reshape(-1, C)
        dx.copy_(v.reshape(shp))

    def pool_bnrelu(self, x, scale, shift, pooled, relu=True):
        v = x.to(_DT[0])
        if scale is not None:
            v = v * scale + shift
        if relu:
            v = torch.relu(v)
        pooled.copy_(v.mean(dim=(1, 2)))

    def sgemm(self, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias=None):
        a = A.view(-1)[: (K if ta else M) * lda].view(K if ta else M, lda)
        a = a[:, :M].t() if ta else a[:, :K]
        b = B.view(-1)[: (N if tb else K) * ldb].view(N if tb else K, ldb)
        b = b[:, :K].t() if tb else b[:, :N]
        out = alpha * (a @ b)
        if bias is not None:
            out = out + bias
        cv = C.view(-1)[: M * ldc].view(M, ldc)[:, :N]
        if beta != 0:
            out = out + beta * cv
        cv.copy_(out)

    def softmax_xent(self, logits, labels, grad_scale, dlogits, loss, correct, probs=None):
        lp = torch.log_softmax(logits.to(_DT[0]), dim=1)
        p = lp.exp()
        lab = labels.long()
        loss.copy_(-lp.gather(1, lab[:, None])[:, 0])
        if probs is not None:
            probs.copy_(p)
        if dlogits is not None:
            oh = F.one_hot(lab, logits.shape[1]).to(_DT[0])
            dlogits.copy_((p - oh) * grad_scale)
        if correct is not None:
            correct.copy_((logits.argmax(1) == lab).int())

    def colsum(self, x, out, scale=1.0, accumulate=False):
        s = x.sum(0) * scale
        if accumulate:
            out.add_(s)
        else:
            out.copy_(s)

    def maxpool_fwd(self, x, y, arg, k, stride, pad_h, pad_w, stats=None):
        self._maxpool_fwd(x, y, arg, k, stride, pad_h, pad_w)
        if stats is not None:
            self.bn_stats(y, stats)

    def _maxpool_fwd(self, x, y, arg, k, stride, pad_h, pad_w):
        N, H, W, C = x.shape
        _, P, Q, _ = y.shape
        xc = x.to(_DT[0]).permute(0, 3, 1, 2)
        pb = (P - 1) * stride + k - pad_h - H
        pr = (Q - 1) * stride + k - pad_w - W
        xp = F.pad(xc, (pad_w, pr, pad_h, pb), value=float("-inf"))
        win = xp.unfold(2, k, stride).unfold(3, k, stride)  # N C P Q k k
        flat = win.reshape(N, C, P, Q, k * k)
        v, i = flat.max(-1)
        y.copy_(v.permute(0, 2, 3, 1))
        arg.copy_(i.permute(0, 2, 3, 1).to(torch.uint8))

    def maxpool_bwd(self, dy, arg, dx, k, stride, pad_h, pad_w):
        N, H, W, C = dx.shape
        _, P, Q, _ = dy.shape
        Hp = (P - 1) * stride + k
        Wp = (Q - 1) * stride + k
        acc = torch.zeros(N, max(Hp, H + pad_h), max(Wp, W + pad_w), C, dtype=_DT[0])
        a = arg.long()
        d = dy.to(_DT[0])
        for r in range(k):
            for s in range(k):
                m = (a == r * k + s).to(_DT[0]) * d
                acc[:, r:r + (P - 1) * stride + 1:stride, s:s + (Q - 1) * stride + 1:stride, :] += m
        dx.copy_(acc[:, pad_h:pad_h + H, pad_w:pad_w + W, :])

    def sgd_momentum(self, w, m, g, wb, lr_t, momentum, wd, grad_scale, skip=None):
        if skip is not None and int(skip.reshape(-1)[0]) != 0:
            return
        lr = float(lr_t.reshape(-1)[0])
        gg = g.to(w.dtype) * grad_scale + wd * w
        m.mul_(momentum).add_(gg)
        w.sub_(lr * m)
        if wb is not None and wb.data_ptr() != w.data_ptr():
            wb.copy_(w)

    def cast_bf16(self, x, y):
        y.copy_(x)

    def weight_tflip(self, wb, wt, table, ntab, total):
        arr = table.cpu().numpy().view(TDESC)[:ntab]
        for d in arr:
            src, dst, K, R, S, C = (int(d[k]) for k in ("src", "dst", "K", "R", "S", "C"))
            Ru, Sv, r0, s0, dr, ds = (int(d[k]) for k in ("Ru", "Sv", "r0", "s0", "dr", "ds"))
            w = wb.view(-1)[src:src + K * R * S * C].view(K, R, S, C)
            ridx = torch.tensor([r0 + dr * u for u in range(Ru)])
            sidx = torch.tensor([s0 + ds * v for v in range(Sv)])
            sub = w[:, ridx][:, :, sidx]  # K Ru Sv C
            wt.view(-1)[dst:dst + C * Ru * Sv * K].view(C, Ru, Sv, K).copy_(sub.permute(3, 1, 2, 0))

    def zero_(self, t):
        t.zero_()

    def cifar_augment(self, raw_u8, params_i32, out, pad):
        N, H, W, _ = raw_u8.shape
        img = raw_u8.to(_DT[0])
        res = torch.zeros(N, H, W, out.shape[-1], dtype=_DT[0])
        for n in range(N):
            oy, ox, flip = [int(v) for v in params_i32[n].tolist()]
            padded = F.pad(img[n].permute(2, 0, 1), (pad, pad, pad, pad))
            crop = padded[:, oy:oy + H, ox:ox + W]
            if flip:
                crop = crop.flip(2)
            mean = crop.mean()
            std = crop.std(unbiased=False)
            adj = torch.maximum(std, torch.tensor(1.0 / (crop.numel() ** 0.5)))
            res[n, :, :, :3] = ((crop - mean) / adj).permute(1, 2, 0)
        out.copy_(res)

    def vgg_preprocess(self, packed_u8, desc, out, means):
        from ..data.imagenet import vgg_preprocess_np
        N, OH, OW, _ = out.shape
        d = desc if isinstance(desc, np.ndarray) else desc.cpu().numpy()
        buf = packed_u8.cpu().numpy() if hasattr(packed_u8, "cpu") else packed_u8
        res = torch.zeros(N, OH, OW, out.shape[-1], dtype=_DT[0])
        for i in range(N):
            r = d[i]
            img = buf[int(r["offset"]):int(r["offset"]) + int(r["H"]) * int(r["W"]) * 3].reshape(int(r["H"]), int(r["W"]), 3)
            res[i, :, :, :3] = torch.from_numpy(vgg_preprocess_np(img, int(r["rh"]), int(r["rw"]), int(r["cy"]),
                                                                  int(r["cx"]), int(r["flip"]), OH))
        out.copy_(res)

    def synthetic_images(self, out, seed):
        g = torch.Generator().manual_seed(int(seed))
        out.zero_()
        out[..., :3] = torch.rand(out.shape[:-1] + (3,), generator=g) * 2 - 1
