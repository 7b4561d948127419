"""Fake-cluster tests (the analog of the reference's localhost PS/worker runs,
scripts/submit_mac_dist.sh): gloo backend, world 2 on CPU, one process per rank."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grads_for(spec, N, shard, seed):
    from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
    from distributed_resnet_tensorflow_amd.runtime.executor import Executor
    ex = Executor(spec, N, RefBackend(), "cpu", seed=seed)
    g = torch.Generator().manual_seed(100 + shard)
    ex.images[..., :3] = torch.randn(N, 32, 32, 3, generator=g)
    ex.labels.copy_(torch.randint(0, 10, (N,), generator=g, dtype=torch.int32))
    return ex


def _worker(rank, world, port, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
        from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine
        spec = cifar_resnet_v2(8)
        N = 4
        ex = _grads_for(spec, N, rank, seed=1 + rank)   # different init on purpose: broadcast must fix it
        eng = DataParallelEngine(ex, bucket_mb=0.05, mode=mode)
        assert len(eng.buckets) > 1
        eng.broadcast_parameters()
        # expected: mean over ranks of each rank's local gradient (per-replica BN, reference semantics)
        exp = torch.zeros_like(ex.P.grad)
        for r in range(world):
            e2 = _grads_for(spec, N, r, seed=1)
            e2.forward(True)
            e2.backward()
            exp += e2.P.grad / world
        ex.forward(True)
        eng.begin_step()
        ex.backward()
        g = eng.finish()
        st = eng.stats()
        assert st["comm_exposed_ms"] >= 0 and st["backward_ms"] > 0, st
        if mode == "sync":
            err = ((g / world - exp).norm() / exp.norm()).item()
            w_before = ex.P.master.clone()
            ex.set_lr(0.1)
            ex.apply_gradients(grad_scale=1.0 / world, grad=g)
            out = torch.stack([ex.P.master.sum(), (ex.P.master - w_before).norm()])
            gathered = [torch.zeros_like(out) for _ in range(world)]
            dist.all_gather(gathered, out)
            same = all(torch.allclose(gathered[0], t) for t in gathered)
            q.put((rank, err, same))
        else:
            # delayed mode: first step applies nothing, second step applies step-1's average
            assert float(g.abs().sum()) == 0.0
            ex.forward(True)
            eng.begin_step()
            ex.backward()
            g2 = eng.finish()
            err = ((g2 / world - exp).norm() / exp.norm()).item()
            q.put((rank, err, True))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), False))


@pytest.mark.parametrize("mode,world", [("sync", 2), ("delayed", 2), ("sync", 4)])
def test_allreduce_dp_equals_mean_of_replica_gradients(mode, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, err, same in res:
        assert isinstance(err, float), err
        assert err < 1e-5, (rank, err)
        assert same


def test_bucket_layout_grows_from_the_buffer_start():
    """Buckets tile the flat gradient buffer exactly, at slot (tensor) boundaries, in readiness
    order (end of the buffer first), and grow geometrically from the start so that the bucket
    exposed after the backward pass is small (ImageNet ResNet-50: 25 MB cap, 2 MB first)."""
    from distributed_resnet_tensorflow_amd.models.spec import build_spec
    from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine
    from distributed_resnet_tensorflow_amd.runtime.params import ParamStore
    P = ParamStore(build_spec("imagenet", 50), "cpu", False)
    eng = DataParallelEngine.__new__(DataParallelEngine)
    eng.P = P
    mb = (1 << 20) // 4
    b = eng._make_buckets(25 * mb, 2 * mb)
    assert b[0][1] == P.total and b[-1][0] == 0
    assert all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))
    offs = {s.offset for s in P.slots}
    assert all(lo in offs for lo, _ in b)
    largest = max(s.numel for s in P.slots)
    assert (b[-1][1] - b[-1][0]) <= 2 * mb + largest
    assert (b[-1][1] - b[-1][0]) < 4 * mb        # ~2 MB exposed, not a 25 MB bucket
    assert max(hi - lo for lo, hi in b) < 30 * mb


def test_collective_watchdog_fires_on_stalled_exchange():
    import time
    from distributed_resnet_tensorflow_amd.parallel.watchdog import CollectiveWatchdog

    class _Ev:
        def __init__(self, ok):
            self.ok = ok

        def query(self):
            return self.ok

    msgs = []
    # 1) host blocked inside the exchange (a gloo collective waiting for a dead peer)
    wd = CollectiveWatchdog(0.2, on_timeout=msgs.append, poll_s=0.05)
    wd.arm(7)
    time.sleep(0.6)
    assert wd.fired and "step 7" in msgs[-1] and "host" in msgs[-1]
    wd.close()
    # 2) queued on the device but never completing (an RCCL kernel stuck on a dead peer)
    wd = CollectiveWatchdog(0.2, on_timeout=msgs.append, poll_s=0.05)
    wd.arm(8)
    wd.done(_Ev(False))
    time.sleep(0.6)
    assert wd.fired and "step 8" in msgs[-1] and "device" in msgs[-1]
    wd.close()
    # 3) healthy steps never fire
    n = len(msgs)
    wd = CollectiveWatchdog(0.2, on_timeout=msgs.append, poll_s=0.05)
    for step in range(5):
        wd.arm(step)
        wd.done(_Ev(True))
        time.sleep(0.1)
    time.sleep(0.4)
    assert not wd.fired and len(msgs) == n
    wd.close()


def _zero1_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
        from distributed_resnet_tensorflow_amd.parallel.engine import DataParallelEngine
        spec = cifar_resnet_v2(8)
        out = {}
        for shard in (False, True):
            ex = _grads_for(spec, 4, rank, seed=1)
            eng = DataParallelEngine(ex, bucket_mb=0.05, shard_optimizer=shard)
            assert eng.zero1 == shard
            if shard:  # every bucket but the one at the buffer end splits into equal shards
                assert sum(eng._sharded(lo, hi) for lo, hi in eng.buckets) >= len(eng.buckets) - 1
                assert eng.buckets[0][1] == ex.P.total and eng.buckets[-1][0] == 0
            eng.broadcast_parameters()
            ex.set_lr(0.1)
            for _ in range(2):
                ex.forward(True)
                eng.begin_step()
                ex.backward()
                eng.apply_gradients(eng.finish(), 1.0 / world)
            eng.gather_state()
            out[shard] = (ex.P.master.clone(), ex.P.momentum.clone())
        rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
        q.put((rank, rel(out[True][0], out[False][0]), rel(out[True][1], out[False][1])))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_optimizer_matches_allreduce_dp(world):
    """ZeRO-1 (reduce-scatter, per-rank SGD shard, all-gather of the weights) trains to the same
    weights and momentum as all-reduce data parallelism over two steps (the second step uses
    weights the first step's gather produced; gather_state completes the stale shards)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_zero1_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ew, em in res:
        assert isinstance(ew, float), ew
        assert ew < 1e-6 and em < 1e-5, (rank, ew, em)


def _agree_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributed_resnet_tensorflow_amd.train.session import agree_ms
        # rank 0 measured the eager step faster, rank 1 the graph step: alone they would split
        mine = [10.0, 11.0] if rank == 0 else [12.0, 9.5]
        eager_ms, graph_ms = agree_ms(mine)
        q.put((rank, eager_ms, graph_ms, "graph" if graph_ms < eager_ms else "eager"))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e), None))


def test_step_mode_trial_agrees_across_ranks():
    """The session's timing trials (eager vs segmented graphs, side stream vs one stream) decide
    from the slowest rank's timings (train/session.py agree_ms): two ranks whose own timings
    disagree take the SAME step mode."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert all(o[1] != "error" for o in out), out
    assert out[0][1:] == out[1][1:] == (12.0, 11.0, "graph"), out
