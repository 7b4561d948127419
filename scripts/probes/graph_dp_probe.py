"""Probe: capture a data-parallel step (bucketed async RCCL all-reduce fired from backward
hooks) in a HIP graph with a single-rank process group, replay, and compare against eager.
Run under torchrun --nproc-per-node 1 on a GPU box."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))  # repo root
import torch
import torch.distributed as dist

from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine
from distributed_resnet_tensorflow_amd.runtime.executor import Executor
from distributed_resnet_tensorflow_amd.runtime.graph import StepGraph


def build(seed):
    ex = Executor(cifar_resnet_v2(20), 32, HipBackend("cuda"), "cuda", seed=seed)
    ex.images.zero_()
    g = torch.Generator().manual_seed(3)
    ex.images[..., :3] = torch.randn(32, 32, 32, 3, generator=g).bfloat16().cuda()
    ex.labels.copy_(torch.randint(0, 10, (32,), generator=g, dtype=torch.int32))
    ex.set_lr(0.05)
    return ex


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    outs = []
    for use_graph in (False, True):
        ex = build(1)
        eng = DataParallelEngine(ex, bucket_mb=0.5)
        eng.broadcast_parameters()

        def step():
            ex.forward(True)
            eng.begin_step()
            ex.backward()
            eng.finish()
            ex.apply_gradients(grad_scale=1.0)

        run = StepGraph(step, warmup=2).replay if use_graph else step
        if not use_graph:
            step(); step()  # same number of warmup steps as the graph path
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        outs.append(ex.P.master.clone())
    err = ((outs[0] - outs[1]).norm() / outs[0].norm()).item()
    print(f"graph-vs-eager DP weights rel err {err:.3e}", flush=True)
    dist.destroy_process_group()
    assert err < 2e-2, err


if __name__ == "__main__":
    main()
