"""Static-plan training executor for ResNet v2 on the gfx950 kernel library.

This is the analog of the TF1 C++ graph executor the reference runs each
``mon_sess.run(train_op)`` (resnet_cifar_main.py:320-321): one training step =
forward + hand-derived backward + fused SGD-momentum, issued as a fixed sequence of kernel
launches over PRE-ALLOCATED buffers (so the whole step is capturable as one HIP graph,
runtime/graph.py). There is no autograd tape: the backward of the pre-activation network is
written out explicitly, which is what lets BatchNorm/ReLU be fused across kernel boundaries:

  forward, per conv: y = conv( relu(bn(x)) ) [+ shortcut]   -- BN-apply+ReLU in the load
      prologue of the consuming 1x1 convs (rewritten in LDS, never written to HBM) or, for BNs
      feeding a 3x3 conv, materialised once by a streaming kernel (bn_policy); residual add +
      the NEXT BN's partial statistics in the epilogue of the producing conv.
  backward, per conv: dgrad as a forward conv of dY with flipped/transposed weights (the
      projection-shortcut dgrad accumulates through the residual epilogue), wgrad recomputes
      relu(bn(x)) in its load prologue, BN-ReLU backward = reduce -> finalize -> apply (+ the
      identity-shortcut gradient fused into the apply).

Gradients land directly in the flat gradient buffer (runtime/params.py) in reverse creation
order; ``grad_ready`` callbacks report the completed suffix so the data-parallel engine can
start bucket all-reduces while earlier layers are still back-propagating.
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Callable, List, Optional

import torch

from ..models.spec import Block, BN, Conv, NetSpec
from ..ops.backend import BnCfin, ConvGeom, OutMap, dgrad_geom, tflip_desc, tflip_table
from .params import ParamStore

BN_DECAY = 0.997     # reference resnet_model_official.py:37
BN_EPSILON = 1e-5    # reference resnet_model_official.py:38


@dataclass
class BNState:
    bn: BN
    gamma: torch.Tensor
    beta: torch.Tensor
    dgamma: torch.Tensor
    dbeta: torch.Tensor
    run_mean: torch.Tensor
    run_var: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor
    mean: torch.Tensor
    invstd: torch.Tensor
    stats: Optional[torch.Tensor] = None  # partial stats of the normalised tensor [G][2][C]
    G: int = 1
    rows: int = 0                          # N*H*W of the normalised tensor
    src: Optional[torch.Tensor] = None     # the raw (pre-BN) tensor
    act: Optional[torch.Tensor] = None     # materialised relu(bn(src)) (materialize_bn mode)
    bacc: Optional[torch.Tensor] = None    # backward sums [R][2][C] (sum g, sum g*xhat)
    bG: int = 1                            # replicas of bacc
    cfin_pub: bool = False                 # consumer-side finalize: the next consumer publishes

    @property
    def ss(self):
        return (self.scale, self.shift)


@dataclass
class DgradPhase:
    """One launch of a data gradient: a stride-1 conv of dY with (sub-)kernel `wt`, written to the
    whole dX (stride-1 convs) or to one output phase of it (stride-2 convs, `out_map`)."""
    wt_shape: tuple
    wt_off: int
    geom: ConvGeom
    out_map: Optional[OutMap]
    wt: Optional[torch.Tensor] = None


@dataclass
class ConvOp:
    conv: Conv
    geom: ConvGeom
    w: torch.Tensor        # compute weights [K,R,S,C]
    dg: List[DgradPhase]   # data-gradient launches (empty for the stem)
    dw: torch.Tensor       # fp32 grad view [K,R,S,C]
    grad_lo: int           # flat offset of this conv's gradient slot
    full_cover: bool = True  # the phases write every dX element


@dataclass
class BlockPlan:
    blk: Block
    x: torch.Tensor                 # block input (raw residual stream)
    bn: List[BNState]               # [bn1, bn2(, bn3)]
    convs: List[ConvOp]             # main path
    proj: Optional[ConvOp]
    hs: List[torch.Tensor]          # raw conv outputs of the main path except the last
    sc: Optional[torch.Tensor]      # projection output
    out: torch.Tensor               # block output
    grad_lo: int                    # lowest flat grad offset written by this block


class Executor:
    GRAD_BUF_MAX = 64     # rotating data-gradient buffers of ImageNet-sized steps (see _alloc)
    def __init__(self, spec: NetSpec, batch: int, backend, device, seed: int = 0,
                 weight_decay: float = 2e-4, momentum: float = 0.9, params: ParamStore | None = None,
                 materialize_bn: Optional[bool] = None):
        self.spec, self.N, self.be = spec, batch, backend
        # fuse each BN's backward reduction into the epilogue of the data-gradient conv feeding it
        self.fuse_bn_bwd = True
        # (The BN backward applied on load by both 1x1 consumers instead of materialised -- the
        # "BNB prologue" -- measured slower: the 1x1 data gradient re-reads its narrow input once
        # per output-channel tile, ResNet-50 bs128 10.74 -> 11.18 ms; removed in round 5.)
        # split-K weight gradients may accumulate with fp32 atomics (the autotuner's choice per
        # layer; the gradients are then zeroed at the start of every backward); not in the
        # bitwise-reproducible mode
        if hasattr(backend, "wgrad_atomic_ok"):
            backend.wgrad_atomic_ok = os.environ.get("DRN_DETERMINISTIC", "0") != "1"
        # debug mode: synchronous finiteness checks after every block (forward and backward)
        self.check_nan = os.environ.get("DRN_CHECK_NAN", "0") == "1"
        # deterministic mode (DRN_DETERMINISTIC=1): bitwise-reproducible steps -- one statistics
        # slot per producer workgroup (no two atomics ever meet) and the unfused BN-backward
        # reduction (the stride-2 data-gradient phases would share slots)
        self.deterministic = os.environ.get("DRN_DETERMINISTIC", "0") == "1"
        if self.deterministic:
            self.fuse_bn_bwd = False
            if hasattr(backend, "autotune"):
                backend.autotune = False  # timing-dependent tile choices change per-tile partial sums
        # (Producer-side finalize variants -- the last-arriving conv workgroup per channel column,
        # or the streaming apply kernels finalizing G == 1 statistics -- measured slower than the
        # consumer-side finalize below (ResNet-50: 12.85 vs 11.78 ms) and were removed.)
        # Consumer-side BN finalize (off only in the deterministic mode): no finalize launches --
        # the kernels CONSUMING a BatchNorm (the fused-prologue 1x1 convs, the materialising
        # apply, the backward apply) derive its parameters from the statistics replicas in their
        # own prologue and the first of them publishes them (ops/backend.py BnCfin). Removes ~98
        # dependent ~6 us launches per ResNet-50 step from the critical path.
        self.cfin = not self.deterministic
        # single-phase strided data gradients zero the other phases in their own epilogue
        self.out_fill = True
        self.device = torch.device(device)
        self.wd, self.mom = weight_decay, momentum
        self.is_hip = backend.name == "hip"
        # weight gradients on a second HIP stream (DRN_WGRAD_STREAM=1): every wgrad (+ its split-K
        # reduction) only feeds the optimizer, so it runs concurrently with the data-gradient /
        # BN-backward chain of the critical path; events guard the gradient buffers it reads.
        # Only weight gradients (conv_wgrad, its own workspace) run there: the split-K conv
        # workspace and tickets of the backend are used by main-stream launches alone.
        # (Forking the projection-shortcut forward conv onto this stream measured neutral; a
        # CU-masked side stream (hipExtStreamCreateWithCUMask) 5 % slower at 64, 128 and 192 of
        # 256 CUs, profiles/r6_experiments.md; both were removed.)
        self.side = None
        # the data-gradient weight refresh after each update on the side stream (eager steps;
        # neutral vs the main stream, profiles/r4_tflip_side_ab.txt)
        self.tflip_side = True
        # gradient-buffer claims skip the cross-queue wait when the reader already finished
        self.claim_query = True
        if self.is_hip and os.environ.get("DRN_WGRAD_STREAM", "1") == "1":
            self.side = torch.cuda.Stream(self.device)
        # gradient-buffer reuse guard: id(buffer) -> sequence number of the side-stream weight
        # gradient that last read it; _marks[seq] = event recorded after that weight gradient;
        # the main stream has waited for the side stream up to _synced
        self._pending = {}
        self._marks = {}
        # data parallelism: the stream bucket collectives are issued from (_report)
        self._report_stream = None
        self._reported = False
        # cross-stream ordering goes through a scheduler: torch's stream API, or -- while a native
        # step plan is recorded (runtime/plan.py) -- plan event entries replayed from C++
        from .plan import TorchSched
        self.sched = TorchSched()
        self._wseq = 0
        self._synced = 0
        # a claim that needs a wait waits on the side-stream mark up to claim_span weight
        # gradients AFTER the buffer's reader (still many blocks old, so normally complete when
        # the main stream gets there): it covers the next claims too -- one cross-queue barrier
        # packet per claim_span claims instead of one per data gradient
        self.claim_span = 12  # profiles/r4_claim_span_ab.txt
        # BN-apply+ReLU either fused into every consuming conv's load prologue (recomputed by the
        # forward conv, the projection conv and both weight-gradient convs; the LDS-DMA kernels
        # rewrite each landed stage in LDS before its barrier) or materialised once per BN by a
        # streaming kernel (one extra read + write of the tensor). Policy "1x1" (default on the
        # HIP backend): fuse where every consumer is a 1x1 conv -- each element is rewritten once
        # per consuming tile, and the streaming pass it replaces is pure HBM traffic -- and
        # materialise BNs feeding a 3x3 conv, whose 9 taps would transform every element 9 times.
        # "all" materialises every BN, "none" fuses every BN (DRN_BN_MATERIALIZE).
        if materialize_bn is None:
            policy = os.environ.get("DRN_BN_MATERIALIZE", "1x1" if self.is_hip else "all")
        else:
            policy = "all" if materialize_bn else "none"
        assert policy in ("all", "1x1", "none"), policy
        self.bn_policy = policy
        self.materialize_bn = policy != "none"
        # ... and (policy "1x1") BNs whose 1x1 consumer has >= DRN_BN_MAT_TILES 128-wide output-
        # channel tiles: the fused prologue rewrites every input element once per output tile
        # (and again in the weight gradient), so the bottleneck expansions (128->512, 256->1024,
        # 512->2048: 4-16 tiles) spend more VALU on it than one streaming apply pass costs
        # (ResNet-50 bs128, same box, with the 3M threshold below: tiles 8 10.25-10.31 ms, 16
        # 10.29-10.31, 4 10.38-10.40, off 10.36-10.37 -- profiles/r2_experiments.md)
        self.mat_tiles = 8
        # ... but only BN tensors of >= DRN_BN_MAT_MIN_ELEMS elements: below that a step is
        # launch-latency bound and the extra streaming launch costs more than the 3x3 consumer's
        # in-LDS rewrite (CIFAR ResNet-50 bs 128: 2.45 ms materialised vs 2.33 ms fused; its
        # largest BN input is 128x32x32x16 = 2.1M). 3M: the ImageNet 7x7x512 stage (3.2M at bs128)
        # is materialised -- its 3x3 conv and weight gradient ran 80 / 77 us with the prologue
        self.mat_min_elems = 3_000_000
        # the stem's max-pool backward on the weight-gradient side stream in deferred-tail steps
        # (DRN_POOL_BWD_SIDE=0: on the main stream before the optimizer)
        self.pool_bwd_side = os.environ.get("DRN_POOL_BWD_SIDE", "1") == "1"
        # ... and the optimizer's update of every block but the first starts as soon as the side
        # stream has finished their weight gradients (DRN_EARLY_SGD): on the main stream, in the
        # window where it otherwise idles waiting for the first block's weight gradients
        self.early_sgd = os.environ.get("DRN_EARLY_SGD", "1") == "1"
        self._pre_ev, self._pre_lo = None, 0
        self.fdt = backend.acc_dtype
        self.P = params or ParamStore(spec, self.device, keep_bf16=self.is_hip, seed=seed, dtype=self.fdt)
        self.grad_ready: Optional[Callable[[int], None]] = None
        self._alloc()
        self.sync_weights()

    # ------------------------------------------------------------------------------------------
    # allocation
    # ------------------------------------------------------------------------------------------
    def _act(self, *shape):
        return torch.zeros(*shape, dtype=self.be.act_dtype, device=self.device)

    def _f32(self, *shape):
        return torch.zeros(*shape, dtype=self.fdt, device=self.device)

    def _bn_state(self, bn: BN) -> BNState:
        P = self.P
        rm, rv = P.moving(bn.name)
        return BNState(bn, P.w(f"{bn.name}/gamma"), P.w(f"{bn.name}/beta"), P.g(f"{bn.name}/gamma"),
                       P.g(f"{bn.name}/beta"), rm, rv, self._f32(bn.c), self._f32(bn.c), self._f32(bn.c),
                       self._f32(bn.c))

    def _conv_op(self, c: Conv, wt_descs, wt_off, in_hw: int = 0) -> tuple[ConvOp, int]:
        P = self.P
        name = f"{c.name}/kernel"
        s = P.by_name[name]
        g = ConvGeom(c.stride, c.pad, c.pad, 1)
        phases = []
        full = True
        K, R, C = c.cout, c.k, c.cin_store
        if c is not self.spec.stem:
            if c.stride == 1:
                wt_descs.append(tflip_desc(s.offset, wt_off, K, R, R, C))
                phases.append(DgradPhase((C, R, R, K), wt_off, dgrad_geom(g, R, R), None))
                wt_off += s.numel
            else:
                # phase decomposition of the transposed conv: output parity (ph, pw) only sees the
                # taps r = ph + pad (mod 2), at dY offsets d = (ph + pad - r) / 2
                st, p = c.stride, c.pad
                for ph in range(st):
                    rs = [r for r in range(R) if (r - ph - p) % st == 0]
                    for pw in range(st):
                        ss = [q for q in range(R) if (q - pw - p) % st == 0]
                        Hph = (in_hw - ph + st - 1) // st
                        Wph = (in_hw - pw + st - 1) // st
                        if not rs or not ss or Hph <= 0 or Wph <= 0:
                            full = False
                            continue
                        r0, s0 = max(rs), max(ss)
                        dmin_h, dmin_w = (ph + p - r0) // st, (pw + p - s0) // st
                        wt_descs.append(tflip_desc(s.offset, wt_off, K, R, R, C, Ru=len(rs), Sv=len(ss),
                                                   r0=r0, s0=s0, dr=-st, ds=-st))
                        phases.append(DgradPhase((C, len(rs), len(ss), K), wt_off,
                                                 ConvGeom(1, -dmin_h, -dmin_w, 1), OutMap(Hph, Wph, st, ph, pw)))
                        wt_off += C * len(rs) * len(ss) * K
        op = ConvOp(c, g, P.compute_w(name), phases, P.g(name), s.offset, full)
        return op, wt_off

    def _bn_shapes(self):
        """(rows, channels) of every statistics accumulator the plan allocates (upper bound)."""
        sp, N = self.spec, self.N
        hs = sp.stem_hw
        out = [(N * hs * hs, sp.stem.cout)]
        if sp.maxpool:
            out.append((N * sp.pool_hw * sp.pool_hw, sp.stem.cout))
        for blk in sp.blocks:
            hw = blk.in_hw
            out.append((N * hw * hw, blk.in_c))              # bn1 backward sums
            for b, c in zip(blk.bns, blk.convs[:-1]):
                hw = c.out_hw(hw)
                out += [(N * hw * hw, c.cout)] * 2           # forward + backward sums
            out.append((N * blk.out_hw * blk.out_hw, blk.out_c))
        out.append((N * sp.blocks[-1].out_hw ** 2, sp.final_c))
        return out

    def _det_replicas(self, M: int, C: int) -> int:
        """Deterministic mode: one replica per producer workgroup (the most workgroups any conv
        tile config or BN reduction launches for an M x C tensor), so every accumulator slot
        receives exactly one atomic add and the finalize sums the slots in a fixed order."""
        return max(((M + 63) // 64) * ((C + 63) // 64), 1024)

    def _reps(self, C: int) -> int:
        """Atomic-spreading replicas of a C-channel statistics accumulator: the backend's count up
        to 256 channels, fewer for wide BNs (whose producers have few pixel tiles, and whose
        consumers re-read all 2*R*C sums in every workgroup's finalize prologue)."""
        r = max(1, min(self.stats_rep, self.stats_rep * 256 // C))
        return min(r, 8) if self.cfin else r   # the finalizing consumers sum at most 8 replicas

    def _stats_for(self, M: int, C: int) -> tuple[torch.Tensor, int]:
        """A [R][2][C] statistics accumulator (R = the backend's atomic-spreading replicas)
        carved from the per-step-cleared arena."""
        R = self._det_replicas(M, C) if self.deterministic else self._reps(C)
        n = (2 * C * R + 15) // 16 * 16
        if self._arena_off + n > self._arena_cap:
            raise RuntimeError("statistics arena exhausted")
        t = self.stats_arena[self._arena_off:self._arena_off + 2 * C * R].view(R, 2, C)
        self._arena_off += n
        return t, R

    def all_bn_states(self) -> List[BNState]:
        """Every BatchNorm of the network in TF creation order."""
        return [b for bp in self.blocks for b in bp.bn] + [self.final_bn]

    def _alloc(self):
        sp, N = self.spec, self.N
        be = self.be
        # one arena for every BN statistics accumulator (forward sums and backward sums), cleared
        # by a single fill at the start of each training step
        all_c = [b.c for blk in sp.blocks for b in [blk.bn1] + list(blk.bns)] + [sp.final_bn.c, sp.stem.cout]
        self.stats_rep = int(getattr(be, "stats_replicas", 1))
        if self.deterministic:
            arena = 64 + sum(2 * ((2 * c * self._det_replicas(m, c) + 15) // 16 * 16) for m, c in self._bn_shapes())
        else:
            arena = sum(2 * ((2 * c * self._reps(c) + 15) // 16 * 16) for c in all_c) + 64
        self._arena_cap = arena
        self.stats_arena = self._f32(arena)
        self._arena_off = 0
        wt_descs, wt_off = [], 0
        self.stem_op, wt_off = self._conv_op(sp.stem, wt_descs, wt_off)
        # the stem's weights lead the flat parameter buffer: [0, _stem_hi) is the slice the
        # optimizer updates last when backward(defer_tail=True) (0: layout differs, no deferral)
        self._stem_hi = int(self.stem_op.dw.numel()) if self.stem_op.grad_lo == 0 else 0
        # DRN_DEFER_TAIL=auto: only where the stem's weight gradient is long enough to hide the
        # optimizer (ImageNet: 40 G MAC, ~0.2 ms); a CIFAR stem's is microseconds and the split
        # update only adds a launch to its launch-bound graph
        stem_macs = N * sp.stem_hw * sp.stem_hw * sp.stem.cout * sp.stem.k * sp.stem.k * sp.stem.cin_store
        mode = os.environ.get("DRN_DEFER_TAIL", "auto")
        if mode == "0" or (mode == "auto" and stem_macs < 1e9):
            self._stem_hi = 0
        self._tail_ev = None
        self._stem_ev = None   # side stream: the stem's weight gradient (issued last) is done
        self._tflip_ev = None  # side stream: the data-gradient weights of the next backward are ready
        img = sp.image_size
        self.images = self._act(N, img, img, sp.stem.cin_store)
        # Packed stem (csrc/kernels/stem.hip, on the HIP backend): the 7x7/2 stem over
        # RGB runs on a 4-channel copy of the images with a zero pixel column on each side and on
        # weights padded to 8 taps per row, so one 16-byte piece is a tap PAIR: 4 forward k-stages
        # instead of 7 and 2 weight-gradient k-tiles instead of 4 (62.5 % of the 8-channel
        # reduction is zero padding). Checkpoint / optimizer layout is unchanged: the packed
        # weights are derived after every update, the gradient mapped back after the wgrad.
        c0 = sp.stem
        self.stem_pack = (self.is_hip and c0.k % 2 == 1
                          and c0.stride == 2 and c0.cin <= 4 and c0.cin_store == 8 and img % 2 == 0)
        if self.stem_pack:
            s8 = c0.k + 1
            n_xp = N * img * (img + 2) * 4
            # + slack: a tap-pair piece at the last pad column reads 8 bytes past the last row
            self._stem_xp_buf = torch.zeros(n_xp + 64, dtype=torch.bfloat16, device=self.device)
            self.stem_xp = self._stem_xp_buf[:n_xp].view(N, img, img + 2, 4)
            self.stem_w4 = torch.zeros(c0.cout, c0.k, s8, 4, dtype=torch.bfloat16, device=self.device)
            self.stem_dw4 = torch.zeros(c0.cout, c0.k, s8, 4, dtype=torch.float32, device=self.device)
            g0 = self.stem_op.geom
            self.stem_geom4 = ConvGeom(g0.stride, g0.pad_h, g0.pad_w - 1, 1)
        self.labels = torch.zeros(N, dtype=torch.int32, device=self.device)
        hs = sp.stem_hw
        # fused stem conv + max-pool (DRN_STEM_POOL=0: the conv and pooling kernels separately):
        # the ImageNet stem geometry (7x7/2 packed, 3x3/2 pool without leading pad)
        self.stem_pool = (self.stem_pack and sp.maxpool and c0.k == 7 and hs % 16 == 0 and hs <= 112
                          and c0.cout % 32 == 0 and sp.pool_hw == (hs + 1) // 2
                          and max((sp.pool_hw - 1) * 2 + 3 - hs, 0) // 2 == 0 and 0 <= self.stem_geom4.pad_w <= 2 and self.stem_geom4.pad_h <= 3
                          and os.environ.get("DRN_STEM_POOL", "1") == "1")
        self.stem_out = self._act(N, hs, hs, sp.stem.cout)
        max_act = N * hs * hs * sp.stem.cout
        max_bn_part = 0
        if sp.maxpool:
            ph = sp.pool_hw
            self.pool_out = self._act(N, ph, ph, sp.stem.cout)
            self.pool_arg = torch.zeros(N, ph, ph, sp.stem.cout, dtype=torch.uint8, device=self.device)
            self.pool_stats, self.pool_G = self._stats_for(N * sp.pool_hw * sp.pool_hw, sp.stem.cout)
            x, x_stats, x_G = self.pool_out, self.pool_stats, self.pool_G
            self.stem_stats, self.stem_G = None, 0
        else:
            self.stem_stats, self.stem_G = self._stats_for(N * hs * hs, sp.stem.cout)
            x, x_stats, x_G = self.stem_out, self.stem_stats, self.stem_G
        self.blocks: List[BlockPlan] = []
        ws_need = be.wgrad_ws_elems(N * hs * hs, sp.stem.cout, sp.stem.k, sp.stem.k, sp.stem.cin_store)
        if self.stem_pack:  # the packed stem's gradient has fewer k-tiles, so it may take more splits
            ws_need = max(ws_need, be.wgrad_ws_elems(N * hs * hs, *self.stem_dw4.shape))
        for blk in sp.blocks:
            bns = [self._bn_state(blk.bn1)] + [self._bn_state(b) for b in blk.bns]
            bns[0].stats, bns[0].G = x_stats, x_G
            bns[0].rows = x.numel() // blk.in_c
            bns[0].src = x
            convs = []
            h_in = blk.in_hw
            for c in blk.convs:
                op, wt_off = self._conv_op(c, wt_descs, wt_off, in_hw=h_in)
                convs.append(op)
                h_in = c.out_hw(h_in)
            proj = None
            if blk.proj is not None:
                proj, wt_off = self._conv_op(blk.proj, wt_descs, wt_off, in_hw=blk.in_hw)
            # main-path intermediate outputs + their stats (feeding bn2/bn3)
            h_list = []
            hw = blk.in_hw
            for i, c in enumerate(blk.convs[:-1]):
                hw = c.out_hw(hw)
                h = self._act(N, hw, hw, c.cout)
                st, G = self._stats_for(N * hw * hw, c.cout)
                bns[i + 1].stats, bns[i + 1].G = st, G
                bns[i + 1].rows = N * hw * hw
                bns[i + 1].src = h
                h_list.append(h)
                max_act = max(max_act, h.numel())
            ohw = blk.out_hw
            out = self._act(N, ohw, ohw, blk.out_c)
            sc = self._act(N, ohw, ohw, blk.out_c) if proj is not None else None
            max_act = max(max_act, out.numel(), x.numel())
            grad_lo = min([o.grad_lo for o in convs] + ([proj.grad_lo] if proj else []) +
                          [self.P.by_name[f"{b.bn.name}/gamma"].offset for b in bns])
            bp = BlockPlan(blk, x, bns, convs, proj, h_list, sc, out, grad_lo)
            self.blocks.append(bp)
            out_stats, out_G = self._stats_for(N * ohw * ohw, blk.out_c)
            bp.out_stats, bp.out_G = out_stats, out_G
            # wgrad workspaces
            hw = blk.in_hw
            ins = [x] + h_list
            for op, xin in zip(convs, ins):
                o_hw = op.conv.out_hw(xin.shape[1])
                ws_need = max(ws_need, be.wgrad_ws_elems(N * o_hw * o_hw, op.conv.cout, op.conv.k, op.conv.k,
                                                         op.conv.cin_store))
            if proj is not None:
                ws_need = max(ws_need, be.wgrad_ws_elems(N * ohw * ohw, proj.conv.cout, 1, 1, proj.conv.cin_store))
            x, x_stats, x_G = out, out_stats, out_G
        # head
        self.final_bn = self._bn_state(sp.final_bn)
        self.final_bn.stats, self.final_bn.G = x_stats, x_G
        self.final_bn.rows = x.numel() // sp.final_c
        self.final_bn.src = x
        for bp in self.blocks:
            for i, b in enumerate(bp.bn):
                consumers = [bp.convs[i].conv] + ([bp.proj.conv] if i == 0 and bp.proj is not None else [])
                big = b.src.numel() >= self.mat_min_elems

                def fusable(c):
                    return c.k == 1 and -(-c.cout // 128) < self.mat_tiles
                if self.bn_policy == "all" or (self.bn_policy == "1x1" and big and
                                               not all(fusable(c) for c in consumers)):
                    b.act = self._act(*b.src.shape)
        for b in [b for bp in self.blocks for b in bp.bn] + [self.final_bn]:
            b.bacc, b.bG = self._stats_for(b.rows, b.bn.c)
        self.last_out = x
        C, ncls = sp.final_c, sp.num_classes
        self.pooled = self._f32(N, C)
        self.logits = self._f32(N, ncls)
        self.dlogits = self._f32(N, ncls)
        self.loss_vec = self._f32(N)
        self.correct = torch.zeros(N, dtype=torch.int32, device=self.device)
        self.dpool = self._f32(N, C)
        self.dense_w = self.P.w(f"{sp.dense_name}/kernel")
        self.dense_b = self.P.w(f"{sp.dense_name}/bias")
        self.dense_dw = self.P.g(f"{sp.dense_name}/kernel")
        self.dense_db = self.P.g(f"{sp.dense_name}/bias")
        # backward scratch (stream-ordered reuse)
        # A pool of gradient buffers used least-recently-first: a buffer is rewritten only after
        # len(pool) - 2 other gradients were, so the side-stream weight gradient that read it has
        # long finished and the main stream's data-gradient chain does not wait for it (with 3
        # buffers those waits cost ~1.5 ms of main-stream idle per ResNet-50 step). With the
        # critical path on the high-priority stream the side stream runs further behind: ResNet-50
        # bs128, one box, 3 rounds: 6 buffers 10.13-10.22 ms, 16: 10.07-10.13, 24: 10.01-10.05
        # (profiles/r3s2_gradbufs.txt); 32 / 64 / 96: 9.771-9.804 / 9.762-9.780 / 9.755-9.778 ms
        # (profiles/r5_grad_bufs_ab.txt: from 64 on the pool outnumbers the ~50 buffers a ResNet-50
        # backward takes -- the LRU order restarts every step -- so no data gradient waits on a
        # side-stream reader; 96 only adds unused buffers). Default 64 (~13 GB at ResNet-50 bs128
        # of the 288 GB), at most ~8 % of the device memory, for ImageNet-sized activations; small
        # ones (CIFAR: latency-bound
        # kernels on L2-resident tensors, 2.06-2.28 ms with 32 buffers vs 1.8-2.1 ms) keep 6.
        # Data parallelism uses the same pool: a bucket's all-reduce is issued from the side
        # stream right after the bucket's last weight gradient (_report), which is the earliest
        # point its data exists whatever the pool size; the pool only decides how long the
        # critical-path data gradients wait for side-stream readers (single-rank RCCL engine,
        # ResNet-50 bs128: 10.02 ms vs 9.87 ms plain, profiles/r4_base).
        buf_bytes = max_act * torch.finfo(self.be.act_dtype).bits // 8
        if self.side is not None and buf_bytes >= (64 << 20):
            cap = int(0.08 * torch.cuda.get_device_properties(self.device).total_memory) // max(1, buf_bytes) \
                if self.device.type == "cuda" else 32
            nbuf = max(6, min(self.GRAD_BUF_MAX, cap))
        else:
            nbuf = 6 if self.side is not None else 3
        self.g_bufs = [self._act(max_act) for _ in range(nbuf)]
        self.g_a, self.g_b, self.g_c = self.g_bufs[:3]
        self._lru: List[int] = []
        self.bn_part = self._f32(2 * max(b.bn.c for bp in self.blocks for b in bp.bn + [self.final_bn]))
        self.bn_coef = self._f32(3 * max(b.bn.c for bp in self.blocks for b in bp.bn + [self.final_bn]))
        self.wgrad_ws = self._f32(max(ws_need, 16))
        # data-gradient weights (flipped / channel-transposed), one flat buffer + device table
        self.wt_flat = torch.zeros(max(wt_off, 16), dtype=self.be.act_dtype, device=self.device)
        self.wt_descs = wt_descs
        table, nt, total = tflip_table(wt_descs)
        self.wt_table, self.wt_n, self.wt_total = table.to(self.device), nt, total
        for op in self._all_ops():
            for ph in op.dg:
                n = 1
                for d in ph.wt_shape:
                    n *= d
                ph.wt = self.wt_flat[ph.wt_off:ph.wt_off + n].view(ph.wt_shape)
        self.lr_t = self._f32(1)

    def _all_ops(self):
        yield self.stem_op
        for bp in self.blocks:
            yield from bp.convs
            if bp.proj is not None:
                yield bp.proj

    # ------------------------------------------------------------------------------------------
    # weights
    # ------------------------------------------------------------------------------------------
    def sync_weights(self):
        """Refresh the compute copies (bf16 + flipped dgrad weights) from the fp32 master."""
        if self.P.wbf16 is not None:
            self.be.cast_bf16(self.P.master, self.P.wbf16)
        src = self.P.wbf16 if self.P.wbf16 is not None else self.P.master
        if self.wt_n:
            if self.is_hip:
                self.be.weight_tflip(src, self.wt_flat, self.wt_table, self.wt_n, self.wt_total)
            else:
                self.be.weight_tflip(src, self.wt_flat, self.wt_table.cpu(), self.wt_n, self.wt_total)
        self._repack_stem()

    def _repack_stem(self):
        """Packed stem weights [K][7][8][4] from the bf16 compute copy (after every update)."""
        if self.stem_pack:
            self.be.stem_pack_weights(self.stem_op.w, self.stem_w4)

    # ------------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------------
    def _fin_fwd_spec(self, b: BNState, publish: bool) -> BnCfin:
        return BnCfin(b.stats, float(b.rows), b.gamma, beta=b.beta, run_mean=b.run_mean, run_var=b.run_var,
                      scale=b.scale, shift=b.shift, mean=b.mean, invstd=b.invstd, publish=publish,
                      momentum=BN_DECAY, eps=BN_EPSILON)

    def _take_fin(self, b: BNState) -> Optional[BnCfin]:
        """The consumer-side finalize for the next kernel consuming relu(bn(b.src)) through its
        fused prologue: only the first consumer of the step finalizes (and publishes); later ones
        read the published scale/shift."""
        if not b.cfin_pub:
            return None
        b.cfin_pub = False
        return self._fin_fwd_spec(b, publish=True)

    def _bn_fwd(self, b: BNState, train: bool):
        if train and self.cfin and b is not self.final_bn:
            if b.act is not None:  # materialised for a 3x3 consumer: the apply finalizes
                self.be.bn_apply_fin(b.src, b.act, self._fin_fwd_spec(b, publish=True), relu=True)
            else:
                b.cfin_pub = True
            return
        if train:
            self.be.bn_finalize(b.stats, b.G, b.rows, b.gamma, b.beta, b.run_mean, b.run_var, b.scale, b.shift,
                                b.mean, b.invstd, BN_DECAY, BN_EPSILON, update_running=True)
        else:
            self.be.bn_inference(b.gamma, b.beta, b.run_mean, b.run_var, BN_EPSILON, b.scale, b.shift, b.mean,
                                 b.invstd)
        if b.act is not None:
            self.be.bn_apply(b.src, b.act, b.scale, b.shift, relu=True)

    def _cin(self, b: BNState):
        """(tensor, in_bn, in_fin) a conv consuming relu(bn(b.src)) reads."""
        if b.act is not None:
            return b.act, None, None
        return b.src, b.ss, self._take_fin(b)

    def forward(self, train: bool = True):
        """Runs the network on self.images/self.labels; fills loss_vec/correct (and dlogits)."""
        be, sp = self.be, self.spec
        if train:
            be.zero_(self.stats_arena)
        st = self.stem_op
        if self.stem_pool:
            # conv + max-pool + the pooled BN statistics in one kernel: the conv output never
            # reaches HBM (csrc/kernels/stem_pool.hip stem_conv_pool_kernel)
            be.stem_pack_input(self.images, self.stem_xp)
            fused = train and not self.deterministic
            img = sp.image_size
            be.stem_conv_pool(self.stem_xp, self.stem_w4, self.pool_out, self.pool_arg, self.stem_geom4, img, img,
                              sp.stem_hw, sp.stem_hw, stats=self.pool_stats if fused else None)
            if train and not fused:
                be.bn_stats(self.pool_out, self.pool_stats)
        elif self.stem_pack:
            be.stem_pack_input(self.images, self.stem_xp)
            be.conv_fwd(self.stem_xp, self.stem_w4, self.stem_out, self.stem_geom4,
                        stats=self.stem_stats if train else None)
        else:
            be.conv_fwd(self.images, st.w, self.stem_out, st.geom, stats=self.stem_stats if train else None)
        if sp.maxpool and not self.stem_pool:
            ph = sp.pool_hw
            pad = max((ph - 1) * 2 + 3 - sp.stem_hw, 0) // 2
            # the first block's BN statistics come out of the pooling kernel itself (the
            # deterministic mode keeps the separate one-replica-per-block statistics pass)
            fused = train and not self.deterministic
            be.maxpool_fwd(self.stem_out, self.pool_out, self.pool_arg, 3, 2, pad, pad,
                           stats=self.pool_stats if fused else None)
            if train and not fused:
                be.bn_stats(self.pool_out, self.pool_stats)
        for bp in self.blocks:
            self._block_fwd(bp, train)
            if self.check_nan:
                self._check(bp.out, f"forward output of block {bp.blk.stage}.{bp.blk.index}")
        fb = self.final_bn
        self._bn_fwd(fb, train)
        be.pool_bnrelu(self.last_out, fb.scale, fb.shift, self.pooled, relu=True)
        N, C, ncls = self.N, sp.final_c, sp.num_classes
        be.sgemm(0, 1, N, ncls, C, 1.0, self.pooled, C, self.dense_w, C, 0.0, self.logits, ncls, bias=self.dense_b)
        be.softmax_xent(self.logits, self.labels, 1.0 / N, self.dlogits if train else None, self.loss_vec,
                        self.correct)
        if self.check_nan:
            self._check(self.loss_vec, "cross-entropy")

    def _check(self, t: torch.Tensor, what: str):
        """DRN_CHECK_NAN=1 debug mode: synchronous finiteness check naming the failing stage."""
        if not bool(torch.isfinite(t.float()).all()):
            raise FloatingPointError(f"non-finite values in {what}")

    def check_gradients(self):
        """Names every trainable variable whose gradient is not finite (debug mode)."""
        bad = [s.name for s in self.P.slots
               if not bool(torch.isfinite(self.P.grad[s.offset:s.offset + s.numel]).all())]
        if bad:
            raise FloatingPointError(f"non-finite gradients: {bad[:8]}{' ...' if len(bad) > 8 else ''}")

    def _block_fwd(self, bp: BlockPlan, train: bool):
        be = self.be
        bn = bp.bn
        self._bn_fwd(bn[0], train)
        if bp.proj is not None:
            xin, pro, fin = self._cin(bn[0])
            be.conv_fwd(xin, bp.proj.w, bp.sc, bp.proj.geom, in_bn=pro, in_fin=fin)
        for i, op in enumerate(bp.convs):
            last = i == len(bp.convs) - 1
            xin, pro, fin = self._cin(bn[i])
            if last:
                res = bp.sc if bp.proj is not None else bp.x
                be.conv_fwd(xin, op.w, bp.out, op.geom, in_bn=pro, residual=res, in_fin=fin,
                            stats=bp.out_stats if train else None)
            else:
                be.conv_fwd(xin, op.w, bp.hs[i], op.geom, in_bn=pro, in_fin=fin,
                            stats=bn[i + 1].stats if train else None)
                self._bn_fwd(bn[i + 1], train)

    # ------------------------------------------------------------------------------------------
    # backward
    # ------------------------------------------------------------------------------------------
    def _view(self, buf, like):
        return buf[:like.numel()].view(like.shape)

    def _bn_bwd(self, b: BNState, x, dy, dx, add=None, dpool=None, pool_hw=0, reduced=False):
        """dx = BN-ReLU backward of (x -> relu(bn(x))) given dy = d/d relu-output; + add.
        reduced: the producing data-gradient conv already ReLU-masked dy and accumulated the
        per-channel sums into bn_part (fused epilogue), so only finalize + apply remain."""
        be = self.be
        M = x.numel() // b.bn.c
        part = b.bacc
        G = b.bG
        if not reduced:
            G = be.bn_bwd_reduce(dy, dpool, pool_hw, x, b.scale, b.shift, b.mean, b.invstd, part)
        if self.cfin:  # finalize in the apply's prologue; it publishes dgamma / dbeta
            fin = BnCfin(part, float(M), b.gamma, mean=b.mean, invstd=b.invstd, dgamma=b.dgamma, dbeta=b.dbeta,
                         publish=True)
            be.bn_bwd_apply_fin(dy, dpool, pool_hw, x, b.scale, b.shift, fin, add, dx, relu=not reduced)
            return
        coef = self.bn_coef[:3 * b.bn.c]
        be.bn_finalize_bwd(part, G, M, b.gamma, b.invstd, b.dgamma, b.dbeta, coef)
        be.bn_bwd_apply(dy, dpool, pool_hw, x, b.scale, b.shift, b.mean, b.invstd, coef, add, dx,
                        relu=not reduced)

    def backward(self, defer_tail: bool = False):
        """Backward pass into P.grad. defer_tail (single-process steps whose next call is
        apply_gradients): the main stream does NOT wait for the stem's weight gradient here;
        apply_gradients first updates every other parameter concurrently with it, then joins."""
        be, sp = self.be, self.spec
        N, C, ncls = self.N, sp.final_c, sp.num_classes
        if getattr(be, "wgrad_atomic_used", False):
            # weight gradients of layers whose split-K partials are added with atomics
            be.zero_(self.P.grad)
        # dense layer: its weight / bias gradients only feed the optimizer, so with the side
        # stream they run there, off the data-gradient chain
        if self.side is not None:
            self.sched.wait_stream(self.side, torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side):
                be.sgemm(1, 0, ncls, C, N, 1.0, self.dlogits, ncls, self.pooled, C, 0.0, self.dense_dw, C)
                be.colsum(self.dlogits, self.dense_db)
        else:
            be.sgemm(1, 0, ncls, C, N, 1.0, self.dlogits, ncls, self.pooled, C, 0.0, self.dense_dw, C)
            be.colsum(self.dlogits, self.dense_db)
        be.sgemm(0, 0, N, C, ncls, 1.0, self.dlogits, ncls, self.dense_w, C, 0.0, self.dpool, C)
        fb = self.final_bn
        hw = self.last_out.shape[1] * self.last_out.shape[2]
        bufs = self.g_bufs
        self._lru = list(range(len(bufs)))
        d_out = self._view(bufs[self._take(bufs, ())], self.last_out)
        self._bn_bwd(fb, self.last_out, None, d_out, dpool=self.dpool, pool_hw=hw)
        self._report(self.P.by_name[f"{fb.bn.name}/gamma"].offset)
        cur = self._lru[-1]  # index of the buffer holding d_out
        self._pending.clear()
        self._marks.clear()
        self._wseq = self._synced = 0
        if self._tflip_ev is not None:  # the flipped weights refreshed on the side stream
            # (a capture starts after its eager warm-up has synchronized: the event is complete,
            # and a graph may not wait on an event recorded outside it)
            if not (self.is_hip and torch.cuda.is_current_stream_capturing()):
                self.sched.wait(torch.cuda.current_stream(self.device), self._tflip_ev, key="tflip")
            self._tflip_ev = None
        deferred = defer_tail and self.side is not None and self.grad_ready is None and self._stem_hi > 0
        self._pre_ev = None
        for bp in reversed(self.blocks):
            if deferred and self.early_sgd and bp is self.blocks[0] and len(self.blocks) > 1:
                # every gradient at offsets >= the next block's is complete once the side stream
                # gets here: the optimizer may update those while block 0 finishes (apply_gradients)
                self._pre_ev, self._pre_lo = self.sched.record(self.side), self.blocks[1].grad_lo
            cur = self._block_bwd(bp, bufs, cur)
            if self.check_nan:
                self._check(self._view(bufs[cur], bp.x), f"input gradient of block {bp.blk.stage}.{bp.blk.index}")
            self._report(bp.grad_lo)
        d_x0 = self._view(bufs[cur], self.blocks[0].x)
        st = self.stem_op
        pool_bwd = None
        if sp.maxpool:
            k = self._take(bufs, (cur,))
            d_stem = self._view(bufs[k], self.stem_out)
            self._claim(bufs[k])
            ph = sp.pool_hw
            pad = max((ph - 1) * 2 + 3 - sp.stem_hw, 0) // 2

            def pool_bwd():
                be.maxpool_bwd(d_x0, self.pool_arg, d_stem, 3, 2, pad, pad)
            if not (deferred and self.pool_bwd_side):
                pool_bwd()
                pool_bwd = None
        else:
            d_stem = d_x0
        self._tail_ev = None
        if deferred:
            # every weight gradient but the stem's is issued on the side stream: the optimizer
            # may update those while the stem's weight gradient (the last, ~0.2 ms on ImageNet)
            # still runs -- see apply_gradients. With pool_bwd_side the max-pool backward that
            # produces the stem's output gradient runs there too, ahead of it: the optimizer
            # then starts right after the last BatchNorm backward instead of after the pooling's
            # (all three are HBM-bound and share the tail)
            self._tail_ev = self.sched.record(self.side)
        if self.stem_pack:
            if getattr(be, "wgrad_atomic_used", False):
                be.zero_(self.stem_dw4)
            self._wgrad(self.stem_xp, d_stem, self.stem_dw4, self.stem_geom4, pre=pool_bwd,
                        post=lambda: be.stem_unpack_grad(self.stem_dw4, st.dw))
        else:
            self._wgrad(self.images, d_stem, st.dw, st.geom, pre=pool_bwd)
        if self._tail_ev is not None:
            self._stem_ev = self.sched.record(self.side)
        self._report(0)
        if self._tail_ev is None:
            self._join()

    def _report(self, lo: int):
        """grad_ready(lo): every gradient at flat offsets >= lo is issued. With the weight-gradient
        side stream, a report that launches a bucket collective is issued from a dedicated report
        stream that waits on two per-bucket readiness events -- the main stream's (the BN-backward
        applies that published the bucket's dgamma / dbeta) and the side stream's (its weight
        gradients) -- so the collective is ordered after exactly its producers while neither
        compute stream waits for the other (round 4 made the SIDE stream catch up with the main
        stream at every launching report, stalling the next blocks' weight gradients)."""
        if self.grad_ready is None:
            return
        if self.sched.recording and not getattr(self.sched, "native_reports", False):
            self.sched.cut(("report", lo))               # a native plan is cut here: the report
            return                                       # runs from Python at each replay
        if self.side is None:
            self.grad_ready(lo)
            return
        owner = getattr(self.grad_ready, "__self__", None)
        if owner is not None and hasattr(owner, "launches_at") and not owner.launches_at(lo):
            self.grad_ready(lo)                          # (advances the frontier, launches nothing)
            return
        if not getattr(owner, "wants_report_stream", True):
            self.grad_ready(lo)                          # (P2P: its comm stream waits on both streams)
            return
        main = torch.cuda.current_stream(self.device)
        if self._report_stream is None:
            self._report_stream = torch.cuda.Stream(self.device)
        rs = self._report_stream
        self.sched.wait_stream(rs, main)                 # readiness event of the main-stream producers
        self.sched.wait_stream(rs, self.side)            # ... and of the weight gradients
        # (P2P engine under a plan recording: the bucket kernels below are recorded into the plan)
        with torch.cuda.stream(rs):
            self.grad_ready(lo)
        self._reported = True

    # -- weight gradients on the side stream ---------------------------------------------------------
    def _wgrad(self, x, dy, dw, geom, in_bn=None, dy_buf=None, post=None, pre=None):
        """Weight gradient into dw (on the side stream when enabled); pre() / post() run right
        before / after it, on the same stream (the stem's max-pool backward producing dy; the
        packed stem mapping its gradient back to the checkpoint layout)."""
        if self.side is None:
            if pre is not None:
                pre()
            self.be.conv_wgrad(x, dy, dw, geom, in_bn=in_bn, ws=self.wgrad_ws)
            if post is not None:
                post()
            return
        main = torch.cuda.current_stream(self.device)
        self.sched.wait_stream(self.side, main)          # x and dy are complete
        with torch.cuda.stream(self.side):
            if pre is not None:
                pre()
            self.be.conv_wgrad(x, dy, dw, geom, in_bn=in_bn, ws=self.wgrad_ws)
            if post is not None:
                post()
        if dy_buf is not None:                           # the main stream must not overwrite dy early
            self._wseq += 1
            self._marks[self._wseq] = self.sched.record(self.side)
            self._pending[id(dy_buf)] = self._wseq

    def _claim(self, buf):
        """Before the main stream writes a rotating gradient buffer: wait for the side-stream
        weight gradient still reading it."""
        seq = self._pending.pop(id(buf), None)
        if seq is None or seq <= self._synced:
            return                       # an earlier wait already ordered main after that reader
        # (the side stream runs in order: waiting on a later mark covers every earlier reader)
        # (never closer than claim_span marks to the newest one: with a small buffer pool -- CIFAR
        # keeps 6 -- the reader is recent and the wait must not extend to the newest marks)
        target = max(seq, min(seq + self.claim_span, self._wseq - self.claim_span))
        s = max(k for k in self._marks if seq <= k <= target)
        ev = self._marks[s]
        self._synced = s
        for k in [k for k in self._marks if k < s]:
            del self._marks[k]
        # an event that has already completed needs no cross-queue barrier packet; inside a
        # capture the dependency must be recorded as a graph edge regardless
        if self.claim_query and not torch.cuda.is_current_stream_capturing() and self.sched.done(ev):
            return
        self.sched.wait(torch.cuda.current_stream(self.device), ev)

    def _join(self, ev=None):
        if self.side is None:
            return
        main = torch.cuda.current_stream(self.device)
        if self._reported:                               # (a capture must rejoin every forked stream)
            self.sched.wait_stream(main, self._report_stream)
            self._reported = False
        if ev is None:
            self.sched.wait_stream(main, self.side)
            self._pending.clear()
            self._marks.clear()
            self._synced = self._wseq
        else:
            self.sched.wait(main, ev)

    def _dgrad(self, op: ConvOp, dy, dx, accumulate: bool, bn: Optional[BNState] = None, bn_x=None):
        """Data gradient of `op` into dx (+= when accumulate). With bn set (requires a launch set
        covering every dx element) the epilogue also performs that BN's backward reduction."""
        # a single-phase strided data gradient (1x1 stride-2 projection) writes the zeros of the
        # other phases from its own epilogue instead of a separate clearing pass over dx
        fill = self.out_fill and not accumulate and not op.full_cover and len(op.dg) == 1 \
            and op.dg[0].out_map is not None and bn is None
        if not accumulate and not op.full_cover and not fill:
            self.be.zero_(dx)
        fuse = None
        if bn is not None:
            assert op.full_cover
            fuse = (bn_x, bn.scale, bn.shift, bn.mean, bn.invstd)
        for ph in op.dg:
            self.be.conv_fwd(dy, ph.wt, dx, ph.geom, residual=dx if accumulate else None, out_map=ph.out_map,
                             stats=bn.bacc if fuse is not None else None, bn_bwd=fuse, out_fill=fill)

    def _block_bwd(self, bp: BlockPlan, bufs, cur: int) -> int:
        """Back-propagates one block; bufs[cur] holds d(block output). Returns the index of the
        buffer holding d(block input). The dgrad of conv i writes the least recently used buffer
        not holding d(block output) or its dY, and the BN-ReLU backward then runs in place on it."""
        be = self.be
        if len(self._lru) != len(bufs):
            self._lru = list(range(len(bufs)))
        d_out = self._view(bufs[cur], bp.out)
        ins = [bp.x] + bp.hs                 # raw inputs of each main-path conv
        dy, dy_buf, dy_k = d_out, bufs[cur], cur
        for i in reversed(range(len(bp.convs))):
            op, xin, b = bp.convs[i], ins[i], bp.bn[i]
            tgt_k = self._take(bufs, (cur, dy_k))
            tgt = bufs[tgt_k]
            a_in, pro = (b.act, None) if b.act is not None else (b.src, b.ss)
            self._wgrad(a_in, dy, op.dw, op.geom, in_bn=pro, dy_buf=dy_buf)
            if i == 0 and bp.proj is not None:
                self._wgrad(a_in, d_out, bp.proj.dw, bp.proj.geom, in_bn=pro, dy_buf=bufs[cur])
            self._claim(tgt)
            da = self._view(tgt, xin)        # d relu(bn(xin))
            add = None
            fuse = self.fuse_bn_bwd and op.full_cover
            if i == 0 and bp.proj is not None:
                # the projection's data gradient first, the main conv's accumulating one last so
                # that its (full-cover, stride-1) epilogue can carry the fused BN reduction
                pj = bp.proj
                self._dgrad(pj, d_out, da, accumulate=False)
                self._dgrad(op, dy, da, accumulate=True, bn=b if fuse else None, bn_x=xin)
            else:
                self._dgrad(op, dy, da, accumulate=False, bn=b if fuse else None, bn_x=xin)
                if i == 0:
                    add = d_out              # identity shortcut
            self._bn_bwd(b, xin, da, da, add=add, reduced=fuse)
            dy, dy_buf, dy_k = da, tgt, tgt_k
        return dy_k

    def _take(self, bufs, busy) -> int:
        """Index of the least recently used gradient buffer not holding a live gradient (`busy`);
        marks it most recently used."""
        k = next(j for j in self._lru if j not in busy)
        self._lru.remove(k)
        self._lru.append(k)
        return k

    # ------------------------------------------------------------------------------------------
    # optimizer
    # ------------------------------------------------------------------------------------------
    def set_lr(self, lr: float):
        self.be.fill_(self.lr_t, float(lr))

    def join_grads(self):
        """Make the current stream wait for a stem weight gradient deferred by backward() (its
        event only: work queued on the side stream after it -- the data-gradient weight refresh
        -- is not waited for)."""
        if self._tail_ev is not None:
            self._tail_ev = None
            ev, self._stem_ev = self._stem_ev, None
            self._join(ev)

    def apply_gradients(self, grad_scale: float = 1.0, grad: Optional[torch.Tensor] = None,
                        skip: Optional[torch.Tensor] = None):
        """Fused SGD-momentum + weight-layout refresh. skip: optional device int32 word; when it
        is non-zero at run time no parameter or momentum changes (the P2P error word)."""
        P = self.P
        g = P.grad if grad is None else grad
        if self._tail_ev is not None and grad is None:
            # parameters [stem_hi, end) while the stem's weight gradient finishes on the side
            # stream (the stem has no data-gradient weights, so the refresh goes first too)
            hi, ev = self._stem_hi, self._tail_ev
            main = torch.cuda.current_stream(self.device)
            if self._pre_ev is not None and self._pre_lo > hi:
                lo, pre = self._pre_lo, self._pre_ev
                self._pre_ev = None
                self.sched.wait(main, pre)
                wb = P.wbf16[lo:] if P.wbf16 is not None else None
                self.be.sgd_momentum(P.master[lo:], P.momentum[lo:], g[lo:], wb, self.lr_t, self.mom, self.wd,
                                     grad_scale, skip)
                self.sched.wait(main, ev)
                wb = P.wbf16[hi:lo] if P.wbf16 is not None else None
                self.be.sgd_momentum(P.master[hi:lo], P.momentum[hi:lo], g[hi:lo], wb, self.lr_t, self.mom,
                                     self.wd, grad_scale, skip)
            else:
                self._pre_ev = None
                self.sched.wait(main, ev)
                wb = P.wbf16[hi:] if P.wbf16 is not None else None
                self.be.sgd_momentum(P.master[hi:], P.momentum[hi:], g[hi:], wb, self.lr_t, self.mom, self.wd,
                                     grad_scale, skip)
            self.refresh_dgrad_weights(stem=False)  # (the stem's weights are not updated yet)
            self.join_grads()
            wb = P.wbf16[:hi] if P.wbf16 is not None else None
            self.be.sgd_momentum(P.master[:hi], P.momentum[:hi], g[:hi], wb, self.lr_t, self.mom, self.wd,
                                 grad_scale, skip)
            self._repack_stem()
            return
        self.join_grads()
        self.be.sgd_momentum(P.master, P.momentum, g, P.wbf16, self.lr_t, self.mom, self.wd, grad_scale, skip)
        self.refresh_dgrad_weights()

    def sgd_range(self, lo: int, hi: int, grad_scale: float, grad: Optional[torch.Tensor] = None):
        """Fused SGD-momentum on the flat slice [lo, hi) only (sharded optimizer)."""
        P = self.P
        g = P.grad if grad is None else grad
        wb = P.wbf16[lo:hi] if P.wbf16 is not None else None
        self.be.sgd_momentum(P.master[lo:hi], P.momentum[lo:hi], g[lo:hi], wb, self.lr_t, self.mom, self.wd,
                             grad_scale)

    def refresh_dgrad_weights(self, stem: bool = True):
        """Rebuild the flipped / channel-transposed data-gradient weights (and the packed stem's
        weights) from the compute copy. Eager steps with the side stream run the rebuild there:
        only the NEXT backward's data gradients read these weights, so it overlaps the next
        forward pass instead of sitting between the update and the next step (the backward waits
        for its event). A captured step keeps it on the capturing stream (a graph must rejoin
        every forked stream before it ends)."""
        P = self.P
        if self.wt_n:
            src = P.wbf16 if P.wbf16 is not None else P.master
            table = self.wt_table if self.is_hip else self.wt_table.cpu()
            if self.side is not None and self.tflip_side and not torch.cuda.is_current_stream_capturing():
                self.sched.wait_stream(self.side, torch.cuda.current_stream(self.device))  # the updated weights
                with torch.cuda.stream(self.side):
                    self.be.weight_tflip(src, self.wt_flat, table, self.wt_n, self.wt_total)
                self._tflip_ev = self.sched.record(self.side, key="tflip")
            else:
                self.be.weight_tflip(src, self.wt_flat, table, self.wt_n, self.wt_total)
        if stem:
            self._repack_stem()

    def autotune(self):
        """Run one forward + backward so the backend times and fixes its kernel configurations
        (conv tile / pipeline choice per geometry) before graph capture or any collective; the
        BN moving statistics and gradients are restored afterwards (no training side effects)."""
        saved = self.P.bn_state.clone()
        hook, self.grad_ready = self.grad_ready, None
        side, self.side = self.side, None  # time candidate kernels on an otherwise idle GPU
        self.forward(train=True)
        self.backward()
        self.side = side
        self.grad_ready = hook
        self.P.bn_state.copy_(saved)
        self.P.grad.zero_()
        if self.is_hip:
            torch.cuda.synchronize()
            self.insitu_tune(rounds=int(os.environ.get("DRN_INSITU_ROUNDS", "2")))
            if hasattr(self.be, "save_tune_db"):
                self.be.save_tune_db()   # persist newly timed kernel choices (ops/tunedb.py)

    def insitu_tune(self, rounds: int = 2):
        """Re-time the autotuner's finalists of every forward / data-gradient conv INSIDE real
        forward + backward passes (weight gradients running beside them on the side stream, the
        operands as the previous kernel left them in the caches) and keep, per geometry, the one
        with the least in-step time. The isolated tuner times a kernel re-launched on L2-warm
        operands on an idle GPU; in the step some layers ran ~30 % slower than their isolated
        time, and not always with the same ranking. Events bracket each conv launch only while
        this runs; BN moving statistics and gradients are restored afterwards."""
        be = self.be
        cands = {k: v for k, v in getattr(be, "conv_cands", {}).items() if len(v) > 1}
        if not cands:
            return
        saved = self.P.bn_state.clone()
        hook, self.grad_ready = self.grad_ready, None
        width = max(len(v) for v in cands.values())
        best = {k: {} for k in cands}
        for _ in range(rounds):
            for r in range(width):
                for k, v in cands.items():
                    be.conv_cfg[k] = v[r % len(v)]
                be._insitu = []
                try:
                    self.forward(train=True)
                    self.backward()
                    torch.cuda.synchronize()
                    sums = {}
                    for key, cfg, e0, e1 in be._insitu:
                        if key in best:
                            sums[(key, cfg)] = sums.get((key, cfg), 0.0) + e0.elapsed_time(e1)
                finally:
                    be._insitu = None
                for (key, cfg), ms in sums.items():
                    best[key][cfg] = min(best[key].get(cfg, float("inf")), ms)
        changed = 0
        for k, times in best.items():
            pick = min(times.items(), key=lambda kv: kv[1])[0] if times else cands[k][0]
            changed += pick != cands[k][0]
            be.conv_cfg[k] = pick
            if hasattr(be, "tune_db"):
                be.tune_db().put_conv(k, pick)
        be.insitu_changed = changed
        be.conv_cands = {}
        self.grad_ready = hook
        self.P.bn_state.copy_(saved)
        self.P.grad.zero_()
        torch.cuda.synchronize()

    def train_step(self, lr: Optional[float] = None, grad_scale: float = 1.0, allreduce: Optional[Callable] = None):
        if lr is not None:
            self.set_lr(lr)
        self.forward(train=True)
        self.backward(defer_tail=allreduce is None and not self.check_nan)
        if self.check_nan:
            self.check_gradients()
        if allreduce is not None:
            allreduce()
        self.apply_gradients(grad_scale)

    # ------------------------------------------------------------------------------------------
    # metrics (host side, off the hot path)
    # ------------------------------------------------------------------------------------------
    def metrics(self) -> dict:
        xent = float(self.loss_vec.double().mean())
        prec = float(self.correct.double().mean())
        l2 = float(self.P.trainable_l2())
        return {"cross_entropy": xent, "cost": xent + self.wd * l2, "precision": prec}
