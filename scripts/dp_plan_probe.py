#!/usr/bin/env python3
"""Host-side breakdown of a data-parallel native-plan replay over RCCL on one GPU (single-rank
process group): time per step in the native segments, the bucket reports (collective issue),
begin_step / finish, against the eager step and the device time.

    python scripts/dp_plan_probe.py [--dataset cifar10] [--batch 32] [--steps 50]
"""
import argparse
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="cifar10")
    ap.add_argument("--resnet_size", type=int, default=50)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--bucket_mb", type=float, default=25.0)
    ap.add_argument("--pg_first", type=int, default=0, help="create the process group before the priority stream")
    a = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29541"),
                      RANK="0", WORLD_SIZE="1")
    os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    torch.cuda.set_device(0)
    from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine, use_priority_main_stream
    if not a.pg_first:
        use_priority_main_stream()
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    if a.pg_first:
        use_priority_main_stream()
    from distributed_resnet_tensorflow_amd.models.spec import build_spec
    from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
    from distributed_resnet_tensorflow_amd.runtime.executor import Executor
    from distributed_resnet_tensorflow_amd.runtime.plan import StepPlan
    spec = build_spec(a.dataset, a.resnet_size)
    be = HipBackend("cuda")
    ex = Executor(spec, a.batch, be, "cuda", seed=1, weight_decay=2e-4)
    eng = DataParallelEngine(ex, bucket_mb=a.bucket_mb, allreduce="rccl")
    be.synthetic_images(ex.images, seed=17)
    ex.labels.copy_(torch.randint(0, spec.num_classes, (a.batch,), dtype=torch.int32))
    ex.set_lr(0.1)
    ex.autotune()

    def eager():
        ex.forward(train=True)
        eng.begin_step()
        ex.backward()
        eng.apply_gradients(eng.finish(), 1.0)

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    print(f"buckets {len(eng.buckets)}: {[hi - lo for lo, hi in eng.buckets]}", flush=True)
    print(f"eager step {timed(eager, a.steps):.3f} ms", flush=True)
    plan = StepPlan(ex, eng, grad_scale=1.0, warmup=1)
    print(f"plan stats {plan.stats()}", flush=True)
    print(f"plan step {timed(plan.replay, a.steps):.3f} ms", flush=True)

    # instrumented replay: host time per kind of action
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    L, p = plan.L, plan.p

    def replay_instr():
        begin = 0
        for end, action in plan.cuts:
            if end > begin:
                t = time.perf_counter()
                L.drn_plan_replay(p, begin, end)
                acc["native segments"] += time.perf_counter() - t
                cnt["native segments"] += 1
            begin = end
            if action is None:
                continue
            t = time.perf_counter()
            if action == "begin":
                eng.begin_step()
                k = "begin_step"
            elif action == "finish":
                eng.finish()
                k = "finish"
            else:
                launches = eng.launches_at(action[1])
                ex._report(action[1])
                k = "report (launches a bucket)" if launches else "report (no bucket)"
            acc[k] += time.perf_counter() - t
            cnt[k] += 1

    replay_instr()
    torch.cuda.synchronize()
    acc.clear()
    cnt.clear()
    t = time.perf_counter()
    for _ in range(a.steps):
        replay_instr()
    host = (time.perf_counter() - t) / a.steps * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / a.steps * 1e3
    print(f"instrumented replay: host {host:.3f} ms/step, wall {wall:.3f} ms/step", flush=True)
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:30s} {v / a.steps * 1e3:8.3f} ms/step  ({cnt[k] // a.steps} per step)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
