"""SessionRunHook analogs (reference resnet_cifar_main.py:270-307, resnet_imagenet_main.py:207-261).

  LoggingHook     LoggingTensorHook: step / loss / precision / lr every N steps (CIFAR 20,
                  ImageNet 40) + throughput (images/sec, steps/sec) — the reference has no timer
                  (SURVEY Q17); optional metrics.jsonl.
  SummaryHook     SummarySaverHook(save_steps=100): cross_entropy, cost, learning_rate,
                  Precision (+ images/sec) as tfevents (chief only).
  CheckpointHook  MonitoredTrainingSession(save_checkpoint_secs=60) saver (chief only).
  StopAtStepHook  StopAtStepHook(last_step=train_steps) (the reference CIFAR main never stops:
                  SURVEY Q5; here --train_steps is honoured).
  FaultInjectHook test hook: hard-exits one rank at a given step (restart/resume tests).
  ProfileHook     roctx ranges (one per step, and the data / fwd / bwd / comm / optimizer phases
                  inside it) + torch.profiler trace for --profile_steps=a:b.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Optional

log = logging.getLogger("drn")


class Hook:
    def begin(self, sess):
        pass

    def before_step(self, sess, step: int):
        pass

    def after_step(self, sess, step: int, metrics_fn):
        """step = global step AFTER the update; metrics_fn() fetches loss/precision (syncs)."""
        pass

    def end(self, sess):
        pass

    def should_stop(self, step: int) -> bool:
        return False


class LoggingHook(Hook):
    def __init__(self, every_n: int, batch_per_step: int, metrics_path: Optional[str] = None, with_lr: bool = True,
                 world: int = 1):
        self.n = max(1, every_n)
        self.bps = batch_per_step
        self.world = max(1, world)
        self.metrics_path = metrics_path
        self.with_lr = with_lr
        self._t = None
        self._s = None

    def begin(self, sess):
        self._t, self._s = time.time(), sess.global_step

    def after_step(self, sess, step, metrics_fn):
        if step % self.n:
            return
        m = metrics_fn()
        now = time.time()
        dt = max(now - self._t, 1e-9)
        steps = step - self._s
        m["steps_per_sec"] = steps / dt
        m["images_per_sec"] = steps * self.bps / dt
        m["images_per_sec_per_gpu"] = m["images_per_sec"] / self.world
        self._t, self._s = now, step
        parts = [f"step = {step}", f"loss = {m['cost']:.5f}", f"precision = {m['precision']:.5f}"]
        if self.with_lr:
            parts.append(f"lr = {m['learning_rate']:.5g}")
        parts.append(f"({m['steps_per_sec']:.2f} steps/sec, {m['images_per_sec']:.1f} images/sec)")
        if "comm_exposed_ms" in m:
            parts.append(f"[allreduce exposed {m['comm_exposed_ms']:.2f} ms"
                         + (f", overlap {m['overlap_fraction']:.0%}" if "overlap_fraction" in m else "") + "]")
        log.info(", ".join(parts))
        if self.metrics_path:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps({"step": step, "time": now, **m}) + "\n")


class SummaryHook(Hook):
    def __init__(self, writer, every_n: int = 100):
        self.w = writer
        self.n = max(1, every_n)

    def after_step(self, sess, step, metrics_fn):
        if step % self.n:
            return
        m = metrics_fn()
        self.w.add_scalars(step, {"cross_entropy": m["cross_entropy"], "cost": m["cost"],
                                  "learning_rate": m["learning_rate"], "Precision": m["precision"]})

    def end(self, sess):
        self.w.flush()


class CheckpointHook(Hook):
    """Time-based checkpoints (MonitoredTrainingSession save_checkpoint_secs) + one at the end.
    `agree` (sharded optimizer: the hook runs on every rank and the save is collective) turns the
    chief's timer decision into every rank's decision."""
    writes_checkpoint = True  # skipped by the session's end-of-run after a failed step

    def __init__(self, save_secs: float, save_fn, agree=None):
        self.secs = save_secs
        self.save_fn = save_fn
        self.agree = agree
        self._last = None
        self._last_step = -1

    def begin(self, sess):
        self._last = time.time()

    def after_step(self, sess, step, metrics_fn):
        due = self.secs > 0 and time.time() - self._last >= self.secs
        if self.agree is not None:
            due = self.agree(due)
        if due:
            self.save_fn(step, blocking=False)
            self._last = time.time()
            self._last_step = step

    def end(self, sess):
        if sess.global_step != self._last_step:
            self.save_fn(sess.global_step, blocking=True)


class StopAtStepHook(Hook):
    def __init__(self, last_step: Optional[int]):
        self.last = last_step

    def should_stop(self, step):
        return self.last is not None and step >= self.last


class FaultInjectHook(Hook):
    def __init__(self, step: int, rank: int, my_rank: int):
        self.step, self.rank, self.me = step, rank, my_rank

    def after_step(self, sess, step, metrics_fn):
        if self.step >= 0 and step == self.step and self.me == self.rank:
            marker = os.environ.get("DRN_FAULT_MARKER")
            if marker:
                if os.path.exists(marker):
                    return  # already injected once (restarted run continues)
                open(marker, "w").write(str(step))
            log.error("fault injection: rank %d exiting at step %d", self.me, step)
            os._exit(17)


class ProfileHook(Hook):
    """--profile_steps=a:b -> roctx range per step (visible to rocprofv3 --marker-trace) and a
    torch.profiler chrome trace of steps a..b in <logdir>/profile."""

    def __init__(self, spec: str, logdir: str):
        a, b = spec.split(":")
        self.a, self.b = int(a), int(b)
        self.logdir = logdir
        self.prof = None
        from ..utils import profiler
        self.roctx = profiler.Roctx()
        profiler.enable_phases(True)  # data / fwd / bwd / comm / optimizer ranges inside each step

    def before_step(self, sess, step):
        if step == self.a:
            import torch
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts)
            self.prof.__enter__()
        if self.a <= step <= self.b:
            self.roctx.push(f"step {step}")

    def after_step(self, sess, step, metrics_fn):
        if self.a < step <= self.b + 1:
            self.roctx.pop()
        if self.prof is not None and step > self.b:
            self.prof.__exit__(None, None, None)
            os.makedirs(os.path.join(self.logdir, "profile"), exist_ok=True)
            self.prof.export_chrome_trace(os.path.join(self.logdir, "profile", f"trace_{self.a}_{self.b}.json"))
            self.prof = None
