"""Training session: the MonitoredTrainingSession analog (reference resnet_cifar_main.py:309-337).

restore-or-init from `checkpoint_dir` (chief restores, then a rank-0 broadcast replaces both
the PS variable fetch and Horovod's BroadcastGlobalVariablesHook), chief-only hooks (summaries,
checkpoints), per-step LR feed, `should_stop()` via hooks, and a final checkpoint on exit.
One step = feeder.next() -> [HIP graph replay | eager fwd/bwd (+ bucketed all-reduce
overlapped with backward) + fused SGD].
"""
from __future__ import annotations

import logging
import os
import time
from typing import Callable, List, Optional

import torch

from ..ckpt.saver import Saver, latest_checkpoint, write_graph_pbtxt
from ..ops.backend import HipBackend, RefBackend
from ..parallel.engine import DataParallelEngine
from ..runtime.executor import Executor
from ..runtime.graph import SegmentedStepGraph, StepGraph
from ..runtime.plan import StepPlan
from ..runtime.state import export_state, import_state
from ..utils.profiler import enable_phases, phase
from .hooks import Hook

log = logging.getLogger("drn")


def make_backend(device: str, precision: str = "bf16"):
    """--precision: bf16 = the gfx950 HIP kernel library (bf16 activations / weights, fp32
    accumulation, fp32 master weights, momentum and BN statistics) -- the only GPU path: the
    product never routes a convolution to a vendor library (MIOpen). fp32 is the CPU reference
    backend (the fp32 PyTorch oracle ops); asking for it on a GPU is an error. CPU runs always
    use the fp32 reference backend."""
    if precision not in ("bf16", "fp32"):
        raise ValueError(f"--precision must be bf16 or fp32, got {precision!r}")
    if str(device).startswith("cuda"):
        if precision == "fp32":
            raise ValueError("--precision=fp32 is the CPU reference path; the GPU path is the bf16 HIP kernel "
                             "library (fp32 accumulation, fp32 master weights)")
        return HipBackend(device)
    return RefBackend("cpu")


def agree_ms(values, group=None):
    """The slowest rank's timings (element-wise MAX over the process group): every rank takes a
    timing-based step-mode decision from the same numbers, so no two ranks end up in different
    step modes (bench.py does the same for its graph / eager choice). Identity without an
    initialised multi-rank group."""
    import torch.distributed as dist
    vals = [float(v) for v in values]
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return vals
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.tolist()


class _LazyGraph:
    """Placeholder graph: its first replay() captures the step (the StepGraph warm-up is that
    real step), later replays run the captured graph."""

    def __init__(self, sess):
        self.sess, self.g = sess, None

    def replay(self):
        if self.g is None:
            self.g = self.sess._on_graph_stream(lambda: StepGraph(self.sess._step_body, warmup=1))
        else:
            self.g.replay()


class TrainingSession:
    def __init__(self, spec, batch: int, cluster, *, weight_decay: float, lr_schedule, checkpoint_dir: str = "",
                 max_to_keep: int = 5, seed: int = 0, use_graph: bool = True, sync_mode: str = "sync",
                 bucket_mb: float = 25.0, meta: Optional[dict] = None, allreduce: str = "rccl", wire: str = "fp32",
                 collective_timeout_s: float = 0.0, precision: str = "bf16", shard_optimizer: bool = False,
                 step_trial: bool = True):
        self.cluster = cluster
        self.spec = spec
        self.device = torch.device(cluster.device)
        self.be = make_backend(cluster.device, precision)
        self.ex = Executor(spec, batch, self.be, self.device, seed=seed, weight_decay=weight_decay)
        self.lr = lr_schedule
        self.meta = meta or {}
        # DRN_FORCE_DP=1: the data-parallel engine on a single-rank process group (profiling the
        # multi-GPU step machinery -- comm streams, HW-queue use -- on one GPU)
        dp = cluster.distributed or os.environ.get("DRN_FORCE_DP") == "1"
        if dp and not cluster.distributed:
            import torch.distributed as dist
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", os.environ.get("DRN_FORCE_DP_PORT", "29541"))
                if self.device.type == "cuda":
                    dist.init_process_group("nccl", rank=0, world_size=1, device_id=self.device)
                else:
                    dist.init_process_group("gloo", rank=0, world_size=1)
        self.dp = dp
        self.engine = DataParallelEngine(self.ex, bucket_mb=bucket_mb, mode=sync_mode, allreduce=allreduce, wire=wire,
                                         timeout_s=collective_timeout_s,
                                         shard_optimizer=shard_optimizer) if dp else None
        self.sharded = self.engine is not None and self.engine.zero1
        self.world = cluster.world
        self.ckpt_dir = checkpoint_dir
        self.saver = Saver(checkpoint_dir, max_to_keep) if (checkpoint_dir and cluster.is_chief) else None
        if self.saver is not None:
            os.makedirs(checkpoint_dir, exist_ok=True)
            tf_vars = [(sl.name, tuple(sl.tf_shape)) for sl in self.ex.P.slots]
            tf_vars += [(f"{b.bn.name}/{k}", (b.bn.c,)) for b in self.ex.all_bn_states()
                        for k in ("moving_mean", "moving_variance")]
            write_graph_pbtxt(checkpoint_dir, tf_vars, self.meta)
        self.data_state = {}
        self.restored_from = None
        self._restore()
        if self.device.type == "cuda" and self.be.name == "hip":
            self.ex.autotune()  # fix kernel configurations before any collective / graph capture
        # one GPU: the whole step is one HIP graph. Data parallel with the P2P all-reduce (every
        # collective is a kernel with device-side flags): also the whole step, comm included, in
        # one graph. Data parallel over RCCL: the chain of per-segment graphs
        # (SegmentedStepGraph) or eager, whichever the first steps measure faster
        # or the native step plan (runtime/plan.py: the eager step replayed from C++, the bucket
        # collectives issued from Python at its cut points), whichever the first steps measure
        # fastest (DRN_DP_GRAPH=auto, the default; 1 / 0 force graphs / eager): ImageNet ResNet-50
        # runs fastest with the eager structure (side-stream weight gradients), CIFAR steps are
        # launch-bound in Python (~260 launches for a ~2 ms step)
        dp_ok = dp and self.engine.mode == "sync" and not self.sharded
        dp_graph = os.environ.get("DRN_DP_GRAPH", "auto")
        hip_cuda = self.device.type == "cuda" and self.be.name == "hip"
        # (step_trial=False: a single-GPU session keeps the whole-step graph without timing it)
        # data parallel over P2P: the whole-step graph and the native plan (P2P kernels recorded,
        # runtime/plan.py) are timed against each other, like the single-GPU step
        p2p_trial = (use_graph and hip_cuda and dp_ok and self.engine.p2p is not None and dp_graph == "auto"
                     and step_trial)
        self.use_graph = use_graph and hip_cuda and (
            (dp_ok and self.engine.p2p is not None and not p2p_trial) or (dp_ok and dp_graph == "1")
            or (not dp and not step_trial))
        # step-mode trial of the RCCL data-parallel step: eager, native plan, segmented graphs;
        # of the single-GPU step: the whole-step graph (then its side-stream trial) or the native
        # plan (ImageNet ResNet-50 bs128: plan 9.75 vs graph 10.52 ms, profiles/r5_bench_modes_v1.jsonl)
        modes = None
        if use_graph and hip_cuda and dp_ok and self.engine.p2p is None and dp_graph == "auto":
            modes = ["eager", "plan", "graph"]
        elif (use_graph and hip_cuda and not dp and step_trial) or p2p_trial:
            # (+ the plan recorded without the weight-gradient side stream: small steps, e.g. CIFAR
            # ResNet-50 bs32: bench 1.59 ms one-stream vs 1.70 ms two-stream plan)
            modes = ["graph", "plan"] + (["plan_one_stream"] if self.ex.side is not None else [])
        self._trial = {"modes": modes, "i": 0, "n": 0, "t0": 0.0, "ms": {}} if modes else None
        self._plan: Optional[StepPlan] = None
        self._plan1: Optional[StepPlan] = None     # (trial candidate: one-stream plan)
        self.graph_choice: Optional[dict] = None
        # single-GPU graph step: its first replays time the step with and without the weight-
        # gradient side stream and keep the faster (CIFAR ResNet-50 bs32: one stream 1.585 ms vs
        # 1.785 ms; ImageNet bs128 and CIFAR bs128: the side stream wins) -- DRN_SIDE_TRIAL=0 off
        self._strial = None
        # (also for the data-parallel P2P graph step: its reductions run on the P2P comm stream
        # either way, only the weight gradients move)
        self._side_trial = ((self.use_graph or self._trial is not None)
                            and (self.engine is None or self.engine.p2p is not None)
                            and self.ex.side is not None and os.environ.get("DRN_SIDE_TRIAL", "1") == "1")
        self.side_choice: Optional[dict] = None
        # graphs are captured and replayed from a NORMAL-priority stream (replay from the high-
        # priority eager stream measured far slower: 19.4 vs 11.2 ms, parallel/engine.py), so when
        # the eager step moves to the high-priority stream below, the segmented-graph candidate of
        # the trial keeps this one
        self._graph_stream = None
        if hip_cuda and (self.use_graph or (modes is not None and "graph" in modes)):
            # whole-step / segmented graphs are captured and replayed from a dedicated normal-
            # priority stream of their own, not from the stream current at init (the process's
            # null stream in the CLI, which the feeder's batch copies and preprocessing queue
            # behind: single-GPU graph trial 5.5-7.2 ms there vs 1.68 ms in bench.py,
            # profiles/r5_cli_step_rate.txt)
            self._graph_stream = torch.cuda.Stream(self.device)
        if not self.use_graph and self.device.type == "cuda" and self.be.name == "hip":
            # eager step (data parallel or not): the critical path on its own high-priority HW
            # queue, ahead of the weight-gradient side stream (ResNet-50 bs128 on one GPU: 9.93 vs
            # 10.17 ms per step, profiles/r3_side_stream_ab.txt)
            from ..parallel.engine import use_priority_main_stream
            use_priority_main_stream()
        self._graph: Optional[StepGraph] = None
        self._metrics_cache = None
        self.cur_lr = float("nan")
        # set when a step's gradient exchange failed: no further checkpoint may be written
        self.failed: Optional[str] = None
        if os.environ.get("DRN_ROCTX") == "1":
            enable_phases(True)

    # -- state -----------------------------------------------------------------------------------
    @property
    def global_step(self) -> int:
        return self.ex.P.global_step

    def _restore(self):
        prefix = latest_checkpoint(self.ckpt_dir) if self.ckpt_dir else None
        if prefix is not None and (self.cluster.is_chief or not self.cluster.distributed):
            tensors = Saver.restore(prefix)
            self.data_state = import_state(self.ex, tensors)
            self.restored_from = prefix
            log.info("Restored %s (global_step %d)", prefix, self.ex.P.global_step)
        if self.engine is not None:
            self.engine.broadcast_parameters()
            if self.cluster.is_chief is False:
                self.data_state = {}

    def save(self, step: Optional[int] = None, blocking: bool = True):
        """Chief writes the checkpoint. With the sharded optimizer every rank must call this (the
        masters / momentum are first all-gathered)."""
        if self.sharded:
            self.engine.gather_state()
        if self.saver is None:
            return None
        if self.failed:
            raise RuntimeError(f"refusing to checkpoint after a failed step: {self.failed}")
        if self.engine is not None:
            self._guard(self.engine.check_errors)  # every queued step's exchange succeeded
        step = self.global_step if step is None else step
        extra = dict(self.data_state)
        tensors = export_state(self.ex, extra)
        path = self.saver.save(step, tensors, self.meta, blocking=blocking)
        log.info("Saving checkpoints for %d into %s", step, path)
        return path

    # -- stepping ----------------------------------------------------------------------------------
    def _on_graph_stream(self, fn):
        """fn() on the normal-priority graph stream, ordered after and before the eager stream's
        work (identity when the step never left that stream)."""
        gs = self._graph_stream
        if gs is None:
            return fn()
        cur = torch.cuda.current_stream(self.device)
        gs.wait_stream(cur)
        with torch.cuda.stream(gs):
            r = fn()
        cur.wait_stream(gs)
        return r

    def will_capture(self) -> bool:
        """Whether the next step() captures a HIP graph (no other thread may then touch the GPU
        in ways a global-mode capture forbids: the feeder's prefetch waits, TrainingSession.run)."""
        if self.ex.check_nan:
            return False
        if self.use_graph and (self._graph is None or (isinstance(self._graph, _LazyGraph) and self._graph.g is None)):
            return True
        tr = self._trial
        return tr is not None and tr["modes"][tr["i"]] == "graph" and self._graph is None

    def _step_body(self):
        ex = self.ex
        with phase("fwd"):
            ex.forward(train=True)
        if self.engine is not None:
            self.engine.begin_step()
            with phase("bwd"):  # (bucket all-reduces are issued from inside the backward pass)
                ex.backward()
            with phase("comm"):
                g = self.engine.finish()
            with phase("optimizer"):
                self.engine.apply_gradients(g, 1.0 / self.world)
        else:
            with phase("bwd"):
                ex.backward(defer_tail=not ex.check_nan)
            with phase("optimizer"):
                ex.apply_gradients()

    def step(self):
        """One synchronous training step on the batch already in ex.images / ex.labels."""
        self.cur_lr = self.lr.lr_for_step()
        self.ex.set_lr(self.cur_lr)
        if self.use_graph and not self.ex.check_nan:  # the debug checks synchronize: no capture
            if self._graph is None:  # warm-up = this real step
                if self.engine is not None and self.engine.p2p is None:
                    self._graph = self._on_graph_stream(
                        lambda: SegmentedStepGraph(self.ex, self.engine, 1.0 / self.world, warmup=1))
                else:
                    self._graph = self._on_graph_stream(lambda: StepGraph(self._step_body, warmup=1))
                    if self._side_trial:
                        # [phase, replays in phase, t0, side ms, (side graph, side stream),
                        #  one-stream graph, one-stream ms]
                        self._strial = ["side", 0, 0.0, 0.0, None, None, 0.0]
            else:
                # (the trial's re-capture is an eager warm-up step: the engine brackets it itself)
                hooks = self.engine is not None and not (isinstance(self._graph, _LazyGraph) and self._graph.g is None)
                if hooks:
                    self.engine.replay_begin()
                with phase("step (graph replay)"):
                    self._on_graph_stream(self._graph.replay)
                if hooks:
                    self.engine.replay_end()
                if self._strial is not None:
                    self._side_trial_tick()
        elif self._trial is not None and not self.ex.check_nan:
            self._trial_step()
        elif self._plan is not None and not self.ex.check_nan:
            self._plan.replay()
        else:
            self._step_body()
        self.lr.after_step(self.ex.P.global_step)
        self.ex.P.global_step += 1
        self._metrics_cache = None
        if self.engine is not None:
            self._guard(self.engine.poll_errors)

    TRIAL_WARM, TRIAL_STEPS = 3, 10

    def _trial_step(self):
        """One REAL training step of the step-mode trial (data parallel over RCCL): per mode --
        eager, native plan, segmented graphs -- TRIAL_WARM + TRIAL_STEPS steps (a plan's or a
        graph's construction step runs the step eagerly first and is one of them); the fastest
        mode by the slowest rank's timings stays on every rank. Every mode launches the same
        kernels in the same order on the same buffers: the choice changes the step time, not the
        numerics. Mode switches synchronize the device (each mode orders its own cross-stream
        events)."""
        tr = self._trial
        mode = tr["modes"][tr["i"]]
        W, K = self.TRIAL_WARM, self.TRIAL_STEPS
        if mode == "plan" and self._plan is None:
            torch.cuda.synchronize(self.device)
            # (single GPU: one host thread per stream issues the replay)
            self._plan = StepPlan(self.ex, self.engine, 1.0 / self.world, warmup=1,
                                  threads=2 if (self.engine is None and self.ex.side is not None) else 1)
            return
        if mode == "plan_one_stream" and self._plan1 is None:
            torch.cuda.synchronize(self.device)
            side, self.ex.side = self.ex.side, None
            try:
                self._plan1 = StepPlan(self.ex, self.engine, 1.0 / self.world, warmup=1)
            finally:
                self.ex.side = side
            return
        if mode == "graph" and self._graph is None:
            torch.cuda.synchronize(self.device)
            if self.engine is None or self.engine.p2p is not None:
                self._graph = self._on_graph_stream(lambda: StepGraph(self._step_body, warmup=1))
            else:
                self._graph = self._on_graph_stream(
                    lambda: SegmentedStepGraph(self.ex, self.engine, 1.0 / self.world, warmup=1))
            return
        n = tr["n"]
        if n == W:
            torch.cuda.synchronize(self.device)
            tr["t0"] = time.perf_counter()
        self._run_mode(mode)
        if n < W + K - 1:
            tr["n"] = n + 1
            return
        torch.cuda.synchronize(self.device)
        tr["ms"][mode] = (time.perf_counter() - tr["t0"]) / K * 1e3
        tr["i"], tr["n"] = tr["i"] + 1, 0
        if tr["i"] < len(tr["modes"]):
            return
        modes = tr["modes"]
        ms = agree_ms([tr["ms"][m] for m in modes], getattr(self.engine, "group", None))  # same mode everywhere
        pick = modes[min(range(len(modes)), key=lambda i: ms[i])]
        self.graph_choice = {f"{m}_ms": round(v, 3) for m, v in zip(modes, ms)}
        graph_name = "segmented graphs" if self.engine is not None and self.engine.p2p is None else "graph"
        self.graph_choice["mode"] = {"graph": graph_name, "plan": "native plan",
                                     "plan_one_stream": "native plan (one stream)"}.get(pick, "eager")
        log.info("%s step: %s -> %s", "data-parallel" if self.engine is not None else "single-GPU",
                 ", ".join(f"{m} {v:.3f} ms" for m, v in zip(modes, ms)), self.graph_choice["mode"])
        torch.cuda.synchronize(self.device)
        if pick != "graph":   # back to the eager structure: drop the graphs, weight gradients on the side stream
            self.ex.side = getattr(self._graph, "side_stream", self.ex.side)
            self._graph = None
        else:
            self.use_graph = True
            if self._side_trial:
                # the whole-step graph: its side-stream trial follows (_side_trial_tick)
                self._strial = ["side", 0, 0.0, 0.0, None, None, 0.0]
        if pick == "plan_one_stream":
            # the step stays on one stream from here on (eager fallbacks included)
            self._plan, self.ex.side = self._plan1, None
        elif pick != "plan":
            self._plan = None
        self._plan1 = None
        self._mode = pick
        self._trial = None

    def _run_mode(self, mode: str):
        if mode == "eager":
            self._step_body()
        elif mode == "plan":
            self._plan.replay()
        elif mode == "plan_one_stream":
            self._plan1.replay()
        elif self.engine is None:
            self._on_graph_stream(self._graph.replay)
        else:
            self.engine.replay_begin()
            self._on_graph_stream(self._graph.replay)
            self.engine.replay_end()

    def _side_trial_tick(self):
        """After each REAL graph-replayed step of the side-stream trial, in three timed phases of
        TRIAL_WARM + TRIAL_STEPS replays: with the side stream, then without it (re-captured: its
        eager warm-up is a real step), then with it again (the side stream's time is the better
        of its two phases: the first phase also absorbs the run's start-up ramp, which biased a
        two-phase trial against it). The one-stream graph is kept only on a clear win."""
        tr = self._strial
        W, K = self.TRIAL_WARM, self.TRIAL_STEPS
        tr[1] += 1
        if tr[1] == W:
            torch.cuda.synchronize(self.device)
            tr[2] = time.perf_counter()
        if tr[1] < W + K:
            return
        torch.cuda.synchronize(self.device)
        ms = (time.perf_counter() - tr[2]) / K * 1e3
        if tr[0] == "side":
            # next step: capture without the side stream (StepGraph's warm-up = that step)
            tr[0], tr[1], tr[3], tr[4] = "noside", 0, ms, (self._graph, self.ex.side)
            self.ex.side = None
            self._graph = _LazyGraph(self)
            return
        side_graph, side_stream = tr[4]
        if tr[0] == "noside":
            # back to the side-stream graph for its second timing
            tr[0], tr[1], tr[5], tr[6] = "side2", 0, self._graph, ms
            self.ex.side = side_stream
            self._graph = side_graph
            return
        side_ms, one_ms = min(tr[3], ms), tr[6]
        side_ms, one_ms = agree_ms([side_ms, one_ms], getattr(self.engine, "group", None))  # same choice on every rank
        keep = one_ms < 0.97 * side_ms   # (a clear win only: a host-bound loop times both alike)
        self.side_choice = {"side_ms": round(side_ms, 3), "one_stream_ms": round(one_ms, 3),
                            "mode": "one stream" if keep else "weight-gradient side stream"}
        log.info("graph step: side stream %.3f ms, one stream %.3f ms -> %s", side_ms, one_ms,
                 self.side_choice["mode"])
        if keep:
            self.ex.side = None
            self._graph = tr[5]
        self._strial = None

    def _guard(self, fn):
        """Run an error check; on failure mark the session failed (no checkpoint after it)."""
        try:
            fn()
        except RuntimeError as e:
            self.failed = str(e)
            log.error("step failed: %s", e)
            raise

    def metrics(self) -> dict:
        """Loss / precision / lr of the last step, plus the gradient exchange's
        timing (backward_ms, comm_exposed_ms, comm_ms + overlap_fraction when the process group
        records collective durations) and HBM usage."""
        if self._metrics_cache is None:
            m = self.ex.metrics()
            m["learning_rate"] = self.cur_lr
            if self.engine is not None:
                m.update(self.engine.stats())
                self._guard(self.engine.check_errors)
            if self.device.type == "cuda":
                free, total = torch.cuda.mem_get_info(self.device)
                m["hbm_used_gb"] = (total - free) / 1e9
                m["hbm_peak_alloc_gb"] = torch.cuda.max_memory_allocated(self.device) / 1e9
            self._metrics_cache = m
        return dict(self._metrics_cache)

    def run(self, feeder, hooks: List[Hook], chief_hooks: List[Hook] = ()):
        hooks = list(hooks) + (list(chief_hooks) if self.cluster.is_chief else [])
        for h in hooks:
            h.begin(self)
        prefetch = getattr(feeder, "prefetch", None)
        # the host load of batch k+1 runs on a worker thread while this thread enqueues step k
        # (a graph launch blocks the caller ~1 ms for a CIFAR step; the feeder's staging copies
        # wait on the event that ends the consumption of the previous batch, so they are
        # stream-ordered whichever thread issues them). A step that captures a graph gets its
        # prefetch inline after it: no second thread may allocate or synchronize during a capture
        pool = None
        if prefetch is not None and self.device.type == "cuda":
            from concurrent.futures import ThreadPoolExecutor
            pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="drn-prefetch")
        pending = None
        try:
            while not any(h.should_stop(self.global_step) for h in hooks):
                if pending is not None:
                    pending.result()
                    pending = None
                with phase("data"):
                    if not feeder.next():
                        break
                self.data_state = feeder.state()
                for h in hooks:
                    h.before_step(self, self.global_step)
                capture = self.will_capture()
                if pool is not None and not capture:
                    pending = pool.submit(prefetch)
                self.step()
                if prefetch is not None and (pool is None or capture):
                    # the host loads batch k+1 while the GPU runs step k (enqueued above)
                    with phase("data prefetch"):
                        prefetch()
                for h in hooks:
                    h.after_step(self, self.global_step, self.metrics)
        finally:
            if pending is not None:
                pending.result()
            if pool is not None:
                pool.shutdown(wait=True)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            for h in hooks:
                if self.failed and getattr(h, "writes_checkpoint", False):
                    log.error("no final checkpoint: %s", self.failed)
                    continue
                h.end(self)
            if self.saver is not None:
                self.saver.wait()
            if self.engine is not None and not self.failed:
                # (after a failed exchange a peer may be gone or still mapping this rank's
                # buffers: leave them to process exit instead of a collective teardown)
                self.engine.close()
