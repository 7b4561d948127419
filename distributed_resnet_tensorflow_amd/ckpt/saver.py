"""Checkpoint manager: TF `checkpoint` state file, model.ckpt-<step>.* rotation, atomic and
asynchronous writes, restore of the full training state.

Reference behaviour: MonitoredTrainingSession(checkpoint_dir=log_root,
save_checkpoint_secs=60) saves `model.ckpt-<global_step>` on the chief (rank 0 under Horovod,
resnet_cifar_main_horovod.py:311), keeps the last 5 (Saver max_to_keep), restores the latest on
(re)start; the eval poller reads `log_root/checkpoint` (resnet_cifar_eval.py:100-109).

Saved variables use TF names and layouts (runtime/params.py: to_tf): every trainable variable,
its `<name>/Momentum` slot, BN `moving_mean`/`moving_variance`, `global_step` (int64), plus
`drn/*` data-iterator state. A `.meta` file is written as a small JSON model description (NOT
a TF MetaGraphDef: there is no graph to serialise). Writes go to temporary names and are
renamed into place; the state file is replaced last, so a crash never leaves a state file
pointing at a partial checkpoint.
"""
from __future__ import annotations

import json
import os
import re
import threading
from typing import Dict, List, Optional

import numpy as np

from .bundle import read_bundle, write_bundle

STATE = "checkpoint"


def _quote(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def write_graph_pbtxt(ckpt_dir: str, variables: List[tuple], meta: Optional[dict] = None) -> str:
    """`graph.pbtxt` in checkpoint_dir (the chief's MonitoredTrainingSession writes the
    GraphDef there at start). There is no TF graph here, so this is a text-format
    GraphDef of the *variables* only -- one VariableV2 node per saved tensor with its TF dtype
    and shape, plus global_step -- enough for tools that list a run's variables; it is not an
    executable graph. variables: [(tf_name, tf_shape)]."""
    def node(name, dtype, shape):
        dims = "".join(f"\n          dim {{\n            size: {d}\n          }}" for d in shape)
        return (f"node {{\n  name: {_quote(name)}\n  op: \"VariableV2\"\n"
                f"  attr {{\n    key: \"dtype\"\n    value {{\n      type: {dtype}\n    }}\n  }}\n"
                f"  attr {{\n    key: \"shape\"\n    value {{\n      shape {{{dims}\n      }}\n    }}\n  }}\n}}\n")
    out = ["# drn: variables-only GraphDef (no executable graph); model: " +
           json.dumps(meta or {}, sort_keys=True) + "\n"]
    out += [node(n, "DT_FLOAT", shp) for n, shp in variables]
    out.append(node("global_step", "DT_INT64", ()))
    out.append("versions {\n  producer: 24\n}\n")
    path = os.path.join(ckpt_dir, "graph.pbtxt")
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write("".join(out))
    os.replace(tmp, path)
    return path


def write_state(ckpt_dir: str, latest: str, all_paths: List[str]):
    lines = [f"model_checkpoint_path: {_quote(latest)}"] + \
            [f"all_model_checkpoint_paths: {_quote(p)}" for p in all_paths]
    tmp = os.path.join(ckpt_dir, STATE + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, os.path.join(ckpt_dir, STATE))


def read_state(ckpt_dir: str) -> Optional[dict]:
    p = os.path.join(ckpt_dir, STATE)
    if not os.path.exists(p):
        return None
    latest, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).replace('\\"', '"').replace("\\\\", "\\")
        if k == "model_checkpoint_path":
            latest = v
        elif k == "all_model_checkpoint_paths":
            allp.append(v)
    if latest is None:
        return None
    return {"model_checkpoint_path": latest, "all_model_checkpoint_paths": allp}


def _abs(ckpt_dir, p):
    return p if os.path.isabs(p) else os.path.join(ckpt_dir, p)


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    """tf.train.latest_checkpoint analog; None if missing or the files are incomplete."""
    st = read_state(ckpt_dir) if ckpt_dir and os.path.isdir(ckpt_dir) else None
    if not st:
        return None
    prefix = _abs(ckpt_dir, st["model_checkpoint_path"])
    if os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001"):
        return prefix
    return None


def step_of(prefix: str) -> int:
    m = re.search(r"-(\d+)$", prefix)
    return int(m.group(1)) if m else 0


class Saver:
    def __init__(self, ckpt_dir: str, max_to_keep: int = 5, basename: str = "model.ckpt"):
        self.dir = ckpt_dir
        self.max_to_keep = max_to_keep
        self.basename = basename
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        os.makedirs(ckpt_dir, exist_ok=True)

    def save(self, step: int, tensors: Dict[str, np.ndarray], meta: Optional[dict] = None,
             blocking: bool = True) -> str:
        """Writes model.ckpt-<step>; async when blocking=False (tensors must be host copies)."""
        self.wait()
        name = f"{self.basename}-{step}"
        if blocking:
            self._write(name, tensors, meta)
        else:
            self._thread = threading.Thread(target=self._bg, args=(name, tensors, meta), daemon=True)
            self._thread.start()
        return os.path.join(self.dir, name)

    def _bg(self, name, tensors, meta):
        try:
            self._write(name, tensors, meta)
        except BaseException as e:  # surfaced on the next wait()
            self._error = e

    def _write(self, name, tensors, meta):
        final = os.path.join(self.dir, name)
        tmp = os.path.join(self.dir, f".tmp-{name}-{os.getpid()}")
        write_bundle(tmp, tensors)
        with open(tmp + ".meta", "w") as f:
            json.dump({"format": "drn-meta-v1 (not a TF MetaGraphDef)", **(meta or {})}, f)
        for ext in (".data-00000-of-00001", ".index", ".meta"):
            os.replace(tmp + ext, final + ext)
        st = read_state(self.dir)
        allp = [p for p in (st["all_model_checkpoint_paths"] if st else []) if p != name]
        allp.append(name)
        while len(allp) > self.max_to_keep:
            old = allp.pop(0)
            for ext in (".data-00000-of-00001", ".index", ".meta"):
                try:
                    os.remove(_abs(self.dir, old) + ext)
                except FileNotFoundError:
                    pass
        write_state(self.dir, name, allp)

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    @staticmethod
    def restore(prefix: str) -> Dict[str, np.ndarray]:
        return read_bundle(prefix)
