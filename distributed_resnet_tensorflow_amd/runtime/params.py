"""Flat parameter / gradient / optimizer-state storage in TF creation order.

All trainable variables live back to back in ONE fp32 master buffer (plus same-shaped
momentum and gradient buffers), in ``tf.trainable_variables()`` creation order
(SURVEY §5.4), each slot 64-byte aligned. This is what makes the optimizer a single fused
launch (csrc/kernels/sgd.hip), the data-parallel all-reduce a handful of contiguous bucket
slices (parallel/engine.py) and the checkpoint a straight walk of the buffer (ckpt/bundle.py).

Internal layouts differ from TF's on-disk layouts and are converted only at checkpoint time:
  conv kernel   TF HWIO [k,k,cin,cout]   -> internal KRSC [cout,k,k,cin_store] (stem cin 3 -> 8)
  dense kernel  TF [in,out]              -> internal [out,in]
Initialisers follow TF1 defaults used by the reference (resnet_model_official.py:87-91,
tf.layers.dense at :274/:343, batch_normalization at :45-48):
  conv: variance_scaling_initializer() = truncated normal, stddev sqrt(1/fan_in)/0.8796
  dense kernel: glorot_uniform; dense bias: zeros; BN gamma 1, beta 0, moving mean 0, var 1.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ..models.spec import NetSpec

ALIGN = 16  # elements (64 B of fp32, 32 B of bf16)


@dataclass
class Slot:
    name: str          # TF variable name
    tf_shape: tuple
    shape: tuple       # internal shape
    kind: str          # conv | gamma | beta | dense_w | dense_b
    offset: int
    numel: int         # internal element count (incl. stem channel padding)
    owner: object = None


def _round(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _trunc_normal(shape, std, gen):
    t = torch.empty(shape)
    t.normal_(0.0, 1.0, generator=gen)
    # resample outside 2 std (TF truncated_normal)
    for _ in range(8):
        bad = t.abs() > 2
        if not bad.any():
            break
        t[bad] = torch.empty(int(bad.sum())).normal_(0.0, 1.0, generator=gen)
    t.clamp_(-2, 2)
    return t * std


class ParamStore:
    def __init__(self, spec: NetSpec, device, keep_bf16: bool, seed: int = 0, dtype=torch.float32):
        self.spec = spec
        self.device = torch.device(device)
        self.slots: list[Slot] = []
        off = 0
        for name, tf_shape, kind, owner in spec.trainable_variables():
            if kind == "conv":
                shape = (owner.cout, owner.k, owner.k, owner.cin_store)
            elif kind == "dense_w":
                shape = (tf_shape[1], tf_shape[0])
            else:
                shape = tuple(tf_shape)
            n = 1
            for d in shape:
                n *= d
            self.slots.append(Slot(name, tuple(tf_shape), shape, kind, off, n, owner))
            off += _round(n)
        self.total = _round(off)
        self.by_name = {s.name: s for s in self.slots}
        self.dtype = dtype
        f32 = dict(dtype=dtype, device=self.device)
        self.master = torch.zeros(self.total, **f32)
        self.momentum = torch.zeros(self.total, **f32)
        self.grad = torch.zeros(self.total, **f32)
        self.wbf16 = torch.zeros(self.total, dtype=torch.bfloat16, device=self.device) if keep_bf16 else None
        # BN moving statistics (non-trainable), one flat buffer: [mean | var] per BN
        self.bn_slots = {}
        boff = 0
        for bn in spec.batch_norms():
            self.bn_slots[bn.name] = (boff, bn.c)
            boff += 2 * _round(bn.c)
        self.bn_state = torch.zeros(max(boff, ALIGN), **f32)
        self.global_step = 0
        self.initialize(seed)

    # -- views ------------------------------------------------------------------------------
    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        s = self.by_name[name]
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def w(self, name):
        return self.view(self.master, name)

    def g(self, name):
        return self.view(self.grad, name)

    def compute_w(self, name):
        """The weight tensor the kernels read (bf16 copy on GPU, fp32 master on CPU)."""
        return self.view(self.wbf16 if self.wbf16 is not None else self.master, name)

    def moving(self, bn_name):
        off, c = self.bn_slots[bn_name]
        return self.bn_state[off:off + c], self.bn_state[off + _round(c):off + _round(c) + c]

    # -- init -------------------------------------------------------------------------------
    def initialize(self, seed: int = 0):
        gen = torch.Generator().manual_seed(seed)
        host = torch.zeros(self.total, dtype=torch.float64)
        for s in self.slots:
            v = host[s.offset:s.offset + s.numel].view(s.shape)
            if s.kind == "conv":
                c = s.owner
                fan_in = c.k * c.k * c.cin
                std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
                w = _trunc_normal((c.cout, c.k, c.k, c.cin), std, gen)
                v[..., :c.cin] = w
            elif s.kind == "gamma":
                v.fill_(1.0)
            elif s.kind == "dense_w":
                fan_in, fan_out = s.tf_shape
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                v.copy_(torch.rand(s.shape, generator=gen) * 2 * lim - lim)
        self.master.copy_(host)
        self.momentum.zero_()
        self.grad.zero_()
        bs = torch.zeros_like(self.bn_state, device="cpu")
        for name, (off, c) in self.bn_slots.items():
            bs[off + _round(c):off + _round(c) + c] = 1.0
        self.bn_state.copy_(bs)
        self.global_step = 0

    # -- TF-layout export / import (checkpoint) ----------------------------------------------
    def to_tf(self, name: str, buf: torch.Tensor | None = None, dtype=torch.float32) -> torch.Tensor:
        s = self.by_name[name]
        v = self.view(self.master if buf is None else buf, name).detach().cpu().to(dtype)
        if s.kind == "conv":
            c = s.owner
            return v[..., :c.cin].permute(1, 2, 3, 0).contiguous()  # KRSC -> HWIO
        if s.kind == "dense_w":
            return v.t().contiguous()
        return v.clone()

    def from_tf(self, name: str, value: torch.Tensor, buf: torch.Tensor | None = None):
        s = self.by_name[name]
        dst = self.view(self.master if buf is None else buf, name)
        value = torch.as_tensor(value, dtype=self.dtype)
        if s.kind == "conv":
            c = s.owner
            t = torch.zeros(s.shape, dtype=self.dtype)
            t[..., :c.cin] = value.permute(3, 0, 1, 2)
            dst.copy_(t)
        elif s.kind == "dense_w":
            dst.copy_(value.t())
        else:
            dst.copy_(value.reshape(s.shape))

    def trainable_l2(self) -> torch.Tensor:
        """sum(l2_loss(v)) = sum(v^2)/2 over all trainable variables (padding is zero)."""
        # chunked fp32 dot products summed in fp64: no full-size temporaries (the fp64 copy and
        # its square of a 25M-parameter buffer cost ~0.15 s per logged step on the GPU box)
        parts = [torch.dot(c, c).double() for c in self.master.split(1 << 20)]
        return torch.stack(parts).sum() / 2
