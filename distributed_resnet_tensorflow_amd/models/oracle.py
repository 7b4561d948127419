"""Pure-PyTorch autograd oracle of the ResNet v2 network (fp32, NCHW, TF variable layouts).

An independent re-statement of reference resnet_model_official.py:41-366 using stock
``torch.nn.functional`` ops and autograd. It is NOT a training path: the tests use it to
check the hand-derived forward/backward of the static-plan executor (runtime/executor.py)
and the TF-layout checkpoint conversion, layer by layer.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .spec import BN, Conv, NetSpec

_DECAY, _EPS = 0.997, 1e-5


def _conv(x, w_hwio, c: Conv):
    w = w_hwio.permute(3, 2, 0, 1)
    k, s = c.k, c.stride
    if s > 1:  # fixed_padding (reference :53-77) + VALID
        pb = (k - 1) // 2
        pe = k - 1 - pb
        x = F.pad(x, (pb, pe, pb, pe))
        return F.conv2d(x, w, stride=s)
    return F.conv2d(x, w, stride=1, padding=(k - 1) // 2)  # SAME for odd k


def _bn_relu(x, bn: BN, p, state, training):
    rm, rv = state[bn.name]
    y = F.batch_norm(x, rm, rv, p[f"{bn.name}/gamma"], p[f"{bn.name}/beta"], training=training,
                     momentum=1 - _DECAY, eps=_EPS)
    return torch.relu(y)


def _maxpool_same(x, k=3, s=2):
    H = x.shape[2]
    out = (H + s - 1) // s
    total = max((out - 1) * s + k - H, 0)
    pb = total // 2
    pe = total - pb
    x = F.pad(x, (pb, pe, pb, pe), value=float("-inf"))
    return F.max_pool2d(x, k, s)


def forward(spec: NetSpec, p: Dict[str, torch.Tensor], state: Dict[str, tuple], images_nhwc: torch.Tensor,
            training: bool = True) -> torch.Tensor:
    """Logits of the network. `p` maps TF variable names to tensors in TF layout; `state`
    maps BN names to (moving_mean, moving_variance) tensors updated in place when training."""
    x = images_nhwc[..., :spec.in_channels].to(p[f"{spec.stem.name}/kernel"].dtype).permute(0, 3, 1, 2)
    x = _conv(x, p[f"{spec.stem.name}/kernel"], spec.stem)
    if spec.maxpool:
        x = _maxpool_same(x)
    for blk in spec.blocks:
        shortcut = x
        a = _bn_relu(x, blk.bn1, p, state, training)
        if blk.proj is not None:
            shortcut = _conv(a, p[f"{blk.proj.name}/kernel"], blk.proj)
        h = _conv(a, p[f"{blk.convs[0].name}/kernel"], blk.convs[0])
        for b, c in zip(blk.bns, blk.convs[1:]):
            h = _conv(_bn_relu(h, b, p, state, training), p[f"{c.name}/kernel"], c)
        x = h + shortcut
    x = _bn_relu(x, spec.final_bn, p, state, training)
    x = x.mean(dim=(2, 3))
    return x @ p[f"{spec.dense_name}/kernel"] + p[f"{spec.dense_name}/bias"]


def loss_fn(spec, p, state, images, labels, weight_decay=0.0, training=True):
    logits = forward(spec, p, state, images, training)
    xent = F.cross_entropy(logits, labels.long())
    cost = xent
    if weight_decay:
        cost = xent + weight_decay * sum((v * v).sum() / 2 for v in p.values())
    return logits, xent, cost


def params_from_store(store, requires_grad=True) -> Dict[str, torch.Tensor]:
    out = {}
    for s in store.slots:
        t = store.to_tf(s.name, dtype=store.dtype).clone()
        out[s.name] = t.requires_grad_(requires_grad)
    return out


def state_from_store(store) -> Dict[str, tuple]:
    st = {}
    for name in store.bn_slots:
        m, v = store.moving(name)
        st[name] = (m.detach().cpu().clone(), v.detach().cpu().clone())
    return st
