"""Executor <-> checkpoint tensors (TF variable names and layouts).

Names follow tf.layers auto-naming + TF1 optimizer/BN conventions: trainable
`conv2d_7/kernel` (HWIO), `batch_normalization_3/{gamma,beta}`, `dense/{kernel,bias}`, slots
`<var>/Momentum`, non-trainable `batch_normalization_3/{moving_mean,moving_variance}` and
`global_step` (int64 scalar).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

GLOBAL_STEP = "global_step"


def export_state(ex, extra: Optional[Dict[str, int]] = None) -> Dict[str, np.ndarray]:
    P = ex.P
    out: Dict[str, np.ndarray] = {}
    for s in P.slots:
        out[s.name] = P.to_tf(s.name).numpy()
        out[f"{s.name}/Momentum"] = P.to_tf(s.name, buf=P.momentum).numpy()
    for bn in P.bn_slots:
        m, v = P.moving(bn)
        out[f"{bn}/moving_mean"] = m.detach().float().cpu().numpy().copy()
        out[f"{bn}/moving_variance"] = v.detach().float().cpu().numpy().copy()
    out[GLOBAL_STEP] = np.array(P.global_step, dtype=np.int64)
    for k, v in (extra or {}).items():
        out[f"drn/{k}"] = np.array(v, dtype=np.int64)
    return out


def import_state(ex, tensors: Dict[str, np.ndarray], strict: bool = True) -> Dict[str, int]:
    P = ex.P
    missing = []
    for s in P.slots:
        if s.name in tensors:
            P.from_tf(s.name, torch.from_numpy(np.asarray(tensors[s.name])))
        else:
            missing.append(s.name)
        mk = f"{s.name}/Momentum"
        if mk in tensors:
            P.from_tf(s.name, torch.from_numpy(np.asarray(tensors[mk])), buf=P.momentum)
        else:
            P.view(P.momentum, s.name).zero_()
    for bn in P.bn_slots:
        m, v = P.moving(bn)
        for t, key in ((m, "moving_mean"), (v, "moving_variance")):
            k = f"{bn}/{key}"
            if k in tensors:
                t.copy_(torch.from_numpy(np.asarray(tensors[k], dtype=np.float32)).to(t.dtype))
            else:
                missing.append(k)
    if strict and missing:
        raise KeyError(f"checkpoint is missing {len(missing)} variables, e.g. {missing[:3]}")
    P.global_step = int(np.asarray(tensors.get(GLOBAL_STEP, 0)))
    ex.sync_weights()
    return {k[4:]: int(np.asarray(v)) for k, v in tensors.items() if k.startswith("drn/")}
