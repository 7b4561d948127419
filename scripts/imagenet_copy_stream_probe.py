#!/usr/bin/env python3
"""does the ImageNet feeder's H2D copy stream slow the data-parallel step?

The real-data ImageNet CLI is input-bound on these boxes (JPEG decode, ~1k img/s on 8 cores), so
the step is measured with decoded host batches that are ready instantly: one batch of 375x500
RGB images (the typical ImageNet JPEG size) in page-locked memory, handed to the staged
ImagenetFeeder every step (its H2D copy of ~70 MB + the fused VGG preprocess run for real), under
the training session with the single-rank RCCL data-parallel engine (DRN_FORCE_DP=1: comm and
report streams as at N>1). Modes (one process each):

  synthetic   SyntheticFeeder (no copies: the bench's input)
  copystream  ImagenetFeeder with its own H2D copy stream (the shipped ImageNet setting)
  inline      ImagenetFeeder copying on the consuming stream (COPY_STREAM = False)

each under GPU_MAX_HW_QUEUES=4 (HIP's default: the 4th normal-priority stream shares a hardware queue)
and =8 (a queue per stream).

    python scripts/imagenet_copy_stream_probe.py [--steps 80] [--mode M]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class _ReadyLoader:
    """Yields the same decoded, pinned batch forever (host cost ~0)."""

    def __init__(self, batch, seed=0):
        import numpy as np
        import torch
        from distributed_resnet_tensorflow_amd.data import imagenet as inet
        rng = np.random.default_rng(seed)
        h, w = 375, 500
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8).reshape(-1)
        self.packed = torch.empty(batch * img.size, dtype=torch.uint8, pin_memory=True)
        flat = self.packed.numpy()
        self.desc_t = torch.empty(batch * inet.IMG_DESC.itemsize, dtype=torch.uint8, pin_memory=True)
        desc = self.desc_t.numpy().view(inet.IMG_DESC)
        self.labels = torch.empty(batch, dtype=torch.int32, pin_memory=True)
        for i in range(batch):
            flat[i * img.size:(i + 1) * img.size] = img
            rh, rw, cy, cx, flip = inet.draw_geometry(h, w, True, rng)
            desc[i] = (i * img.size, h, w, rh, rw, cy, cx, flip, 0)
            self.labels[i] = int(rng.integers(1, 1001))
        self.n = 0

    def __iter__(self):
        return self

    def __next__(self):
        self.n += 1
        return self.packed, self.desc_t, self.labels

    def state(self):
        return {"data_batch": self.n}

    def close(self):
        pass


def run_mode(mode, steps, batch):
    import torch
    os.environ["DRN_FORCE_DP"] = "1"
    from distributed_resnet_tensorflow_amd.models.spec import build_spec
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import feeder as fd
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.hooks import Hook, StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    torch.cuda.set_device(0)
    sess = TrainingSession(build_spec("imagenet", 50), batch, ClusterInfo(device="cuda:0"), weight_decay=1e-4,
                           lr_schedule=lr_mod.for_dataset("imagenet"), allreduce="rccl")
    if mode == "synthetic":
        feeder = fd.SyntheticFeeder(sess.ex, seed=0)
    else:
        fd.ImagenetFeeder.COPY_STREAM = mode == "copystream"
        feeder = fd.ImagenetFeeder(sess.ex, _ReadyLoader(batch), True)

    class Times(Hook):
        t = {}

        def after_step(self, s, step, metrics_fn):
            if step in (steps - 40, steps):   # the last 40 steps: after the session's step-mode trial
                torch.cuda.synchronize()
                self.t[step] = time.perf_counter()

    th = Times()
    sess.run(feeder, [StopAtStepHook(steps), th])
    ms = (th.t[steps] - th.t[steps - 40]) / 40 * 1e3
    return {"mode": mode, "ms_per_step": round(ms, 3), "graph_choice": sess.graph_choice,
            "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
            "copy_stream": getattr(feeder, "copy_stream", None) is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=90)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--mode", default="")
    a = ap.parse_args()
    if a.mode:
        print(json.dumps(run_mode(a.mode, a.steps, a.batch)), flush=True)
        return
    for m, q in (("synthetic", "4"), ("copystream", "4"), ("inline", "4"), ("copystream", "8"), ("synthetic", "8"),
                 ("copystream", "4"), ("copystream", "8"), ("inline", "4")):
        env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--mode", m, "--steps", str(a.steps),
                              "--batch", str(a.batch)], capture_output=True, text=True, timeout=900, env=env)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else f'{{"mode": "{m}", "error": {json.dumps(out.stderr[-800:])}}}', flush=True)


if __name__ == "__main__":
    main()
