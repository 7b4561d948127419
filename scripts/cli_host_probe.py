#!/usr/bin/env python3
"""Host-time breakdown of the training CLI's step loop (measurement only): wraps the native-plan
replay, the feeder's next/prefetch, the session step and the hooks with wall-clock timers, runs
resnet_cifar_main's cifar_main with the given flags, and prints per-step means at exit.

    python scripts/cli_host_probe.py --num_gpus=1 --train_data_path=... --batch_size=32 ...
"""
import atexit
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_resnet_tensorflow_amd.runtime import plan as plan_mod  # noqa: E402
from distributed_resnet_tensorflow_amd.train import feeder as feeder_mod  # noqa: E402
from distributed_resnet_tensorflow_amd.train import session as session_mod  # noqa: E402
from distributed_resnet_tensorflow_amd.parallel import engine as engine_mod  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()
state = {"on": False}


def timed(cls, name, key):
    fn = getattr(cls, name)

    def wrap(*a, **k):
        if not state["on"]:
            return fn(*a, **k)
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[key] += time.perf_counter() - t
            cnt[key] += 1
    setattr(cls, name, wrap)


orig_step = session_mod.TrainingSession.step


def step(self):
    # time only after the step-mode trial has picked (steady state)
    state["on"] = self._trial is None and self.ex.P.global_step > 40
    t = time.perf_counter()
    orig_step(self)
    if state["on"]:
        acc["session.step"] += time.perf_counter() - t
        cnt["session.step"] += 1
        now = time.perf_counter()
        if state.get("last") is not None:
            acc["loop iteration"] += now - state["last"]
            cnt["loop iteration"] += 1
        state["last"] = now


session_mod.TrainingSession.step = step
timed(plan_mod.StepPlan, "replay", "plan.replay")
seg = collections.defaultdict(float)


def replay_instr(self):
    """StepPlan.replay with per-segment / per-action host timers."""
    L, p, ex, eng = self.L, self.p, self.ex, self.eng
    begin = 0
    for i, (end, action) in enumerate(self.cuts):
        if end > begin:
            t = time.perf_counter()
            L.drn_plan_replay(p, begin, end)
            if state["on"]:
                seg[f"segment {i:2d} ({end - begin} entries)"] += time.perf_counter() - t
        begin = end
        if action is None:
            continue
        t = time.perf_counter()
        if action == "begin":
            eng.begin_step()
        elif action == "finish":
            eng.finish()
        else:
            ex._report(action[1])
        if state["on"]:
            seg[f"action after segment {i:2d}: {action if isinstance(action, str) else 'report'}"] += time.perf_counter() - t
    if eng is None:
        ex._tail_ev = None


if os.environ.get("PROBE_SEGMENTS") == "1":
    plan_mod.StepPlan.replay = replay_instr
    timed(plan_mod.StepPlan, "replay", "plan.replay")
timed(feeder_mod._StagedFeeder, "next", "feeder.next")
timed(feeder_mod._StagedFeeder, "prefetch", "feeder.prefetch (worker thread)")
timed(engine_mod.DataParallelEngine, "begin_step", "engine.begin_step")
timed(engine_mod.DataParallelEngine, "finish", "engine.finish")
timed(engine_mod.DataParallelEngine, "_launch", "engine._launch (collective issue)")
timed(engine_mod.DataParallelEngine, "poll_errors", "engine.poll_errors")


@atexit.register
def report():
    n = max(cnt["session.step"], 1)
    print(f"== host probe: {n} steady-state steps", flush=True)
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:36s} {v / n * 1e3:8.3f} ms/step  ({cnt[k] / n:.1f} calls/step)", flush=True)
    for k, v in sorted(seg.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {k:52s} {v / n * 1e3:8.3f} ms/step", flush=True)


if __name__ == "__main__":
    from distributed_resnet_tensorflow_amd.cli import cifar_main
    sys.exit(cifar_main([sys.argv[0]] + sys.argv[1:]))
