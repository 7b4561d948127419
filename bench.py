#!/usr/bin/env python3
"""Headline benchmark: whole-node training images/sec of ResNet-50 at bs=128 per GPU.

BASELINE.json metric: "images/sec (whole node) ResNet-50 bs=128/GPU at 1/2/4/8 MI355X".
Default config = the reference's ImageNet ResNet-v2-50 (1001 classes, 224x224, bs 128 per
worker -> global 1024 on 8 GPUs, reference README.md:41-46), synthetic data of that shape and
random-init weights (no datasets/checkpoints on the box). A timed step is the full training
step: forward, backward, gradient all-reduce across ranks (RCCL), fused SGD-momentum update
and weight-layout refresh, in bf16 compute with fp32 master weights.
`--dataset cifar10` benchmarks the CIFAR "ResNet-50" (6n+2, n=8) instead.

Launch: `python bench.py --gpus 1 --steps K --warmup W`, or for N>1
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N`.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Reference numbers: ImageNet ResNet-50 img/s. 1 worker bs128 = 0.96 steps/s
# (row 12, ~123 img/s); 8 workers global 1024 = 0.93 steps/s (row 8, ~952 img/s). Intermediate
# N scale row 8's per-GPU rate. CIFAR: 1 GPU 13.94 steps/s x 128 (row 3), 4 ranks 21.82 x 128
# (row 2), 8 ranks 28.66 x 128 (row 7).
BASELINE_IMG_S = {
    "imagenet": {1: 122.9, 2: 2 * 119.0, 4: 4 * 119.0, 8: 952.3},
    "cifar10": {1: 13.94 * 128, 2: None, 4: 21.82 * 128, 8: 28.66 * 128},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dataset", default="imagenet", choices=["imagenet", "cifar10"])
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--width", type=int, default=1, help="bottleneck width multiplier (2 = Wide-ResNet-50-2)")
    ap.add_argument("--batch_size", type=int, default=128, help="per-GPU batch")
    ap.add_argument("--image_size", type=int, default=224,
                    help="ImageNet input size (rehearsals of the ResNet-50 topology at a small shape; not the headline)")
    ap.add_argument("--graph", type=int, default=-1, help="capture the step in a HIP graph (-1: auto)")
    ap.add_argument("--plan", type=int, default=-1,
                    help="native step plan (runtime/plan.py): -1 auto (timed against the other modes), 0 off, 1 force")
    ap.add_argument("--bucket_mb", type=float, default=25.0)
    ap.add_argument("--allreduce", default="auto", choices=["rccl", "p2p", "auto"],
                    help="auto: the one-shot P2P kernel when the whole gradient is <= 64 MB (CIFAR), else RCCL")
    ap.add_argument("--shard_optimizer", type=int, default=0, help="ZeRO-1 sharded optimizer (N > 1)")
    ap.add_argument("--allreduce_wire", default="fp32", choices=["fp32", "bf16"],
                    help="gradient dtype on the wire (bf16: half the all-reduce bytes)")
    args = ap.parse_args()
    # the result line is the ONLY thing on stdout: libraries that print banners there (RCCL's
    # version block at communicator init) are sent to stderr at the file-descriptor level
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import distributed_resnet_tensorflow_amd  # noqa: F401 -- (package-level process settings precede HIP init)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DRN_BENCH_BACKEND=gloo + DRN_BENCH_ONE_DEVICE=1 rehearse the multi-rank code path with every
    # rank on cuda:0 (a one-GPU box); production runs use RCCL, one GPU per rank
    backend = os.environ.get("DRN_BENCH_BACKEND", "nccl")
    if os.environ.get("DRN_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    # DRN_BENCH_DP=1: run the data-parallel engine (single-rank process group) even at N=1, to
    # measure the DP step machinery on one GPU
    force_dp = os.environ.get("DRN_BENCH_DP") == "1"
    if force_dp and world == 1 and "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"),
                          RANK="0", WORLD_SIZE="1")
    from distributed_resnet_tensorflow_amd.models.spec import build_spec
    spec = build_spec(args.dataset, args.resnet_size, width=args.width)
    if args.dataset == "imagenet" and args.image_size != 224:
        from distributed_resnet_tensorflow_amd.models.spec import imagenet_resnet_v2
        spec = imagenet_resnet_v2(args.resnet_size, width=args.width, image_size=args.image_size)
    # the P2P all-reduce (chosen by --allreduce p2p, or auto for <= 64 MB of gradients) runs the
    # data-parallel step as one HIP graph; RCCL data parallelism runs it eagerly
    from distributed_resnet_tensorflow_amd.parallel.engine import p2p_wanted
    p2p = (world > 1 or force_dp) and p2p_wanted(args.allreduce, spec.num_params() * 4, world,
                                                 shard_optimizer=bool(args.shard_optimizer))
    eager_dp = (world > 1 or force_dp) and not p2p
    prio = None
    if (eager_dp or args.graph == 0) and args.graph != 1:
        # eager data-parallel step: its main (critical-path) stream at HIGH priority -- see
        # parallel.engine.use_priority_main_stream
        from distributed_resnet_tensorflow_amd.parallel.engine import use_priority_main_stream
        use_priority_main_stream()
    elif args.graph == -1 and (p2p or not (world > 1 or force_dp)):
        # auto on one GPU: the EAGER candidate runs on a high-priority main stream too (ResNet-50
        # bs128, one box: 9.92-9.94 ms vs 10.15-10.19 ms on the normal-priority stream,
        # profiles/r3_side_stream_ab.txt); the HIP-graph candidate is captured and replayed from
        # a normal-priority stream (replay from a high-priority one measured far slower); the
        # same for the P2P data-parallel step (graph vs eager vs native plan)
        from distributed_resnet_tensorflow_amd.parallel.engine import make_priority_stream
        prio = make_priority_stream()
    if world > 1 or force_dp:
        # per-collective device timing (two events per bucket all-reduce): the JSON line then
        # reports the exchange's total time and its overlap with the backward pass
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
    from distributed_resnet_tensorflow_amd.runtime.executor import Executor
    from distributed_resnet_tensorflow_amd.runtime.graph import SegmentedStepGraph, StepGraph
    from distributed_resnet_tensorflow_amd.runtime.plan import StepPlan
    from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine

    be = HipBackend("cuda")
    wd = 2e-4 if args.dataset == "cifar10" else 1e-4
    ex = Executor(spec, args.batch_size, be, "cuda", seed=1234, weight_decay=wd)
    eng = DataParallelEngine(ex, bucket_mb=args.bucket_mb, allreduce=args.allreduce, wire=args.allreduce_wire,
                             shard_optimizer=bool(args.shard_optimizer)) if (world > 1 or force_dp) else None
    if eng is not None:
        assert (eng.p2p is not None) == p2p, "bench and engine disagree on the P2P all-reduce"
        eng.broadcast_parameters()
    # synthetic data of the benchmark shape: fixed device batch (no host input pipeline)
    be.synthetic_images(ex.images, seed=17 + rank)
    g = torch.Generator(device="cpu").manual_seed(rank)
    ex.labels.copy_(torch.randint(0, spec.num_classes, (args.batch_size,), generator=g, dtype=torch.int32))
    ex.set_lr(0.1)

    def step():
        ex.forward(train=True)
        if eng is not None:
            eng.begin_step()
        ex.backward(defer_tail=eng is None)
        if eng is not None:
            eng.apply_gradients(eng.finish(), 1.0 / world)
        else:
            ex.apply_gradients()

    eager = step
    if prio is not None:
        def eager():
            with torch.cuda.stream(prio):
                step()

    # kernel autotuning pass (one plain forward + backward) before any collective is in flight,
    # so every rank times its candidate kernels on an otherwise idle GPU
    ex.autotune()
    # one GPU: the whole step in one HIP graph. N GPUs: eager by default -- measured on one GPU
    # with the single-rank RCCL engine, eager 11.90 ms vs per-segment graphs (--graph 1,
    # runtime/graph.py SegmentedStepGraph, bucket all-reduces issued between graphs) 12.22 ms:
    # the ~20 graph launches cost more than the host-side kernel launches they replace
    # (the P2P all-reduce is a set of kernels with device-side flags: a data-parallel step on it is
    # captured whole, comm included -- SURVEY §5.8)
    def _time(fn, n=5):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t

    def _agree(ts):
        """Every rank takes the same decision: the slowest rank's timings."""
        if world > 1:
            tt = torch.tensor(ts, dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ts = tt.tolist()
        return ts

    def _pick(cands):
        """{name: fn} -> the fastest (best of 3 interleaved rounds of 5 untimed-for-the-result
        steps each: a single 5-step comparison picked a slower mode once in three runs)."""
        names = list(cands)
        best = [float("inf")] * len(names)
        for _ in range(3):
            for i, k in enumerate(names):
                best[i] = min(best[i], _time(cands[k]))
        best = _agree(best)
        i = min(range(len(names)), key=lambda j: best[j])
        return names[i], {k: round(v / 5 * 1e3, 3) for k, v in zip(names, best)}

    # Step modes (every one runs the same kernels on the same buffers; the choice changes the
    # step time, not the numerics):
    #   eager  -- the Python step, critical path on a high-priority stream;
    #   plan   -- the eager step recorded once and replayed from C++ (runtime/plan.py): same
    #             streams and priorities, a few host calls per step instead of ~340 launches;
    #   graph  -- the whole step as one HIP graph (P2P data parallelism included), optionally
    #             without the weight-gradient side stream (one-stream graph);
    #   segmented -- RCCL data parallelism as a chain of graphs (--graph 1).
    use_graph = args.graph if args.graph >= 0 else int(eng is None or eng.p2p is not None)
    if eng is not None and eng.zero1:
        use_graph = 0
    want_plan = args.plan != 0 and (eng is None or (not eng.zero1 and eng.mode == "sync"))
    cands, mode_times, plan = {}, None, None

    def in_eager_ctx(fn):
        if prio is None:
            return fn
        def f():
            with torch.cuda.stream(prio):
                fn()
        return f

    one_stream = {}   # modes recorded / captured without the weight-gradient side stream
    if use_graph and eng is not None and eng.p2p is None:
        cands["segmented"] = SegmentedStepGraph(ex, eng, 1.0 / world, warmup=1).replay
    elif use_graph:
        cands["graph"] = StepGraph(step, warmup=2).replay
        if ex.side is not None and args.graph == -1:
            # the graph without the weight-gradient side stream (one stream: CIFAR ResNet-50 bs32
            # 1.585 vs 1.785 ms; the side stream wins for larger steps)
            side, ex.side = ex.side, None
            cands["graph_one_stream"] = StepGraph(step, warmup=2).replay
            ex.side = side
            one_stream["graph_one_stream"] = True
    if args.graph != 1 or not cands:
        cands["eager"] = eager
    if want_plan and (args.plan == 1 or "eager" in cands):
        with torch.cuda.stream(prio) if prio is not None else torch.cuda.stream(torch.cuda.current_stream()):
            plan = StepPlan(ex, eng, grad_scale=1.0 / world, warmup=1)
        cands["plan"] = in_eager_ctx(plan.replay)
        if args.plan == 1:
            cands.pop("eager", None)
        if ex.side is not None:
            # the same plan issued by one host thread per stream (StepPlan.set_threads)
            def plan_mt():
                if plan.threads != 2:
                    plan.set_threads(2)
                plan.replay()

            def plan_1t():
                if plan.threads != 1:
                    plan.set_threads(1)
                plan.replay()
            cands["plan"] = in_eager_ctx(plan_1t)
            cands["plan_threads"] = in_eager_ctx(plan_mt)
            if (eng is None or eng.p2p is not None) and args.plan != 1:
                # ... and a plan recorded without the side stream (small steps)
                side, ex.side = ex.side, None
                with torch.cuda.stream(prio) if prio is not None else torch.cuda.stream(torch.cuda.current_stream()):
                    plan1 = StepPlan(ex, eng, grad_scale=1.0 / world, warmup=1)
                ex.side = side
                cands["plan_one_stream"] = in_eager_ctx(plan1.replay)
                one_stream["plan_one_stream"] = True
    mode = next(iter(cands))
    if len(cands) > 1:
        mode, mode_times = _pick(cands)
    if mode == "plan_one_stream":
        plan = plan1
    run = cands[mode]
    use_graph = int(mode in ("graph", "graph_one_stream", "segmented"))
    # host enqueue time of the chosen mode: one step from an idle queue (nothing blocks), and
    # the median over the timed steps (host time per run() call)
    torch.cuda.synchronize()
    t_host = time.perf_counter()
    run()
    t_host = (time.perf_counter() - t_host) * 1e3
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_calls = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tc = time.perf_counter()
        run()
        t_calls.append(time.perf_counter() - tc)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    img_s = args.batch_size * world * args.steps / dt
    loss = float(ex.loss_vec.float().mean())
    in_sync = None
    if world > 1:
        # after the timed region: every replica must hold bit-identical weights (an exact integer
        # checksum of the fp32 masters, gathered from every rank)
        ck = ex.P.master.view(torch.int32).to(torch.int64).sum().reshape(1)
        ck = ck if backend == "nccl" else ck.cpu()
        allck = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(allck, ck)
        in_sync = all(bool(torch.equal(allck[0], c)) for c in allck)
    dp = None
    if eng is not None:
        # data-parallel diagnostics of the last timed step (rank 0's view; comm_exposed_ms = the
        # exchange time left after the backward pass, overlap_fraction = the share of the
        # collectives' device time hidden under it)
        st = eng.stats()
        dp = {"rccl_world": dist.get_world_size(), "backend": dist.get_backend(),
              "allreduce": "p2p" if eng.p2p is not None else "rccl", "buckets": st.get("allreduce_buckets"),
              "bucket_mb": args.bucket_mb, "wire": eng.wire}
        for k in ("backward_ms", "comm_exposed_ms", "comm_ms", "overlap_fraction"):
            if k in st:
                dp[k] = round(float(st[k]), 3)
        if in_sync is not None:
            dp["replicas_in_sync"] = in_sync
        if plan is not None and mode.startswith("plan"):
            # native segments between the engine's Python-issued bucket collectives
            dp["plan_report_cuts"] = sum(1 for _, act in plan.cuts if isinstance(act, tuple))
    if rank == 0:
        base = BASELINE_IMG_S.get(args.dataset, {}).get(world) \
            if (args.width == 1 and args.resnet_size == 50 and spec.image_size in (224, 32)) else None
        model = f"resnet{args.resnet_size}_v2_{args.dataset}" if args.dataset == "imagenet" else \
            f"cifar10_resnet{args.resnet_size}_v2"
        if args.width > 1:
            model = f"wide_resnet{args.resnet_size}_{args.width}_{args.dataset}"
        out = {
            "metric": "images/sec (whole node) ResNet-50 bs=128/GPU"
            if (args.dataset == "imagenet" and args.resnet_size == 50 and args.width == 1 and args.batch_size == 128
                and spec.image_size == 224)
            else f"images/sec (whole node) {model} bs={args.batch_size}/GPU",
            "value": round(img_s, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "steps_per_sec": round(1e3 / ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base, 3) if base else None,
            "dtype": "bf16",
            "data": "synthetic (random-init weights, fixed synthetic batch of the benchmark shape)",
            "config": {"model": model, "global_batch": args.batch_size * world, "per_gpu_batch": args.batch_size,
                       "image_size": spec.image_size, "num_classes": spec.num_classes,
                       "parallelism": f"dp{world}", "hip_graph": bool(use_graph), "step_mode": mode,
                       "wgrad_side_stream": ex.side is not None and mode not in one_stream,
                       "fused_stem_pool": bool(getattr(ex, "stem_pool", False)),
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")},
            "final_loss": round(loss, 4),
            "host_enqueue_ms": round(t_host, 3),
            "host_call_ms_median": round(sorted(t_calls)[len(t_calls) // 2] * 1e3, 3),
        }
        if plan is not None and mode.startswith("plan"):
            out["plan"] = plan.stats()
        if mode_times is not None:
            out["mode_trial_ms"] = mode_times
        if dp is not None:
            out["data_parallel"] = dp
        print(json.dumps(out), file=result_out, flush=True)
    if os.environ.get("DRN_PRINT_TUNE") == "1" and rank == 0:
        for key, cfg, us in be.tune_log:
            print(f"[tune] {key} -> {cfg} ({us} us)", file=sys.stderr)
        print(f"[tune] in-situ re-timing changed {getattr(be, 'insitu_changed', 0)} conv choices", file=sys.stderr)
        print(f"[tune] {be.db_hits} choices from the kernel-selection database", file=sys.stderr)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
