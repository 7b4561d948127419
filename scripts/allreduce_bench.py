#!/usr/bin/env python3
"""All-reduce microbenchmark for the gradient exchange: RCCL
(torch.distributed "nccl") vs the HIP-IPC peer-to-peer kernels (parallel/p2p.py, one-shot and
two-shot) over message sizes, with a correctness check of every result.

  torchrun --nproc-per-node N scripts/allreduce_bench.py [--sizes_kb 64,1024,...] [--iters 20]

One JSON line per (algorithm, size) from rank 0: time per all-reduce (max over ranks), algorithm
bandwidth (bytes / time) and bus bandwidth (2 (W-1)/W x that, the ring-equivalent figure).
Rehearsal on one GPU: DRN_BENCH_BACKEND=gloo DRN_BENCH_ONE_DEVICE=1 (P2P only; every rank on cuda:0).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes_kb", default="64,256,1024,4096,16384,65536")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--algos", default="rccl,p2p1,p2p2,p2p1b,p2p2b",
                    help="p2p1/p2p2: one-/two-shot fp32 wire; p2p1b/p2p2b: bf16 wire")
    ap.add_argument("--graph", type=int, default=1,
                    help="also time the P2P step captured in a HIP graph (device-side latency, the way "
                         "the training step runs it)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if os.environ.get("DRN_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("DRN_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    if "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29541", RANK="0", WORLD_SIZE="1")
    kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
    dist.init_process_group(backend, **kw)
    from distributed_resnet_tensorflow_amd.parallel.p2p import P2PAllReduce

    sizes = [int(s) * 1024 // 4 // 4 * 4 for s in a.sizes_kb.split(",")]
    nmax = max(sizes)
    grad = torch.empty(nmax, device="cuda")
    algos = a.algos.split(",")
    if backend != "nccl":
        algos = [x for x in algos if x != "rccl"]
    p2p = P2PAllReduce(grad) if any(x.startswith("p2p") and not x.endswith("b") for x in algos) else None
    p2pb = P2PAllReduce(grad, wire="bf16") if any(x.startswith("p2p") and x.endswith("b") for x in algos) else None

    def fill(n):
        grad[:n].copy_(torch.arange(n, device="cuda", dtype=torch.float32).remainder_(97) + rank)

    def expected(n):
        return (torch.arange(n, device="cuda", dtype=torch.float32).remainder_(97) * world +
                world * (world - 1) / 2)

    for algo in algos:
        for n in sizes:
            if algo == "rccl":
                def one():
                    dist.all_reduce(grad[:n])
                out = grad
            else:
                pp = p2pb if algo.endswith("b") else p2p
                pp.two_shot_min = 0 if algo.startswith("p2p2") else 1 << 62

                def one(pp=pp):
                    pp.begin_step()
                    pp.reduce_bucket(0, 0, n)
                    pp.end_step()
                out = pp.out
            fill(n)
            one()
            torch.cuda.synchronize()
            ok = bool(torch.allclose(out[:n], expected(n)))
            for _ in range(a.warmup):
                one()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                one()
            torch.cuda.synchronize()
            dt = torch.tensor([(time.perf_counter() - t0) / a.iters], device="cuda")
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            for pp in (p2p, p2pb):
                if pp is not None:
                    pp.check()
            g_us = None
            if a.graph and algo != "rccl":
                # the same step captured in a HIP graph: what the data-parallel training step pays
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(a.iters):
                        one()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                gt = torch.tensor([(time.perf_counter() - t0) / a.iters], device="cuda")
                dist.all_reduce(gt, op=dist.ReduceOp.MAX)
                g_us = round(float(gt.item()) * 1e6, 2)
                ok = ok and bool(torch.allclose(out[:n], expected(n)))
            if rank == 0:
                t = float(dt.item())
                algbw = n * 4 / t / 1e9
                print(json.dumps({"algo": algo, "bytes": n * 4, "world": world, "us": round(t * 1e6, 2),
                                  "graph_us": g_us, "algbw_GBps": round(algbw, 2),
                                  "busbw_GBps": round(algbw * 2 * (world - 1) / max(world, 1), 2), "correct": ok}),
                      flush=True)
    for pp in (p2p, p2pb):
        if pp is not None:
            pp.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
