"""A failed P2P gradient exchange must fail LOUDLY and must not corrupt the model.

Two ranks share cuda:0 over gloo (a one-GPU box) and train a CIFAR ResNet through the real
TrainingSession with the one-shot P2P all-reduce (parallel/p2p.py, csrc/kernels/allreduce_p2p.hip).
After two good steps and a checkpoint, rank 1 fails:

  * "withhold": rank 1 runs its next (eager) step but never publishes bucket 0
    (DRN_FAULT_P2P_WITHHOLD semantics), then stops -- a rank stuck mid-exchange;
  * "stall": rank 1 simply stops stepping while rank 0 replays its captured whole-step HIP graph.

Rank 0 must then (1) raise out of TrainingSession.run within a few device timeouts
(DRN_P2P_TIMEOUT_MS = 1000), i.e. exit non-zero, (2) leave its fp32 master weights and momentum
bitwise equal to the post-step-2 values (the optimizer kernel reads the exchange's error word and
applies nothing), and (3) write no checkpoint after step 2. The reference has no failure
handling at all (SyncReplicas stalls forever, resnet_model.py:108-116).
"""
import os
import socket
import sys
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flush(q):
    """Queue.put hands the item to a feeder thread; os._exit right after it can kill the process
    before the item reaches the pipe, so close the queue and join that thread first."""
    q.close()
    q.join_thread()


def _worker(rank, mode, port, ck, q, stop):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DRN_P2P_TIMEOUT_MS="1000")
    import torch.distributed as dist
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.feeder import SyntheticFeeder
    from distributed_resnet_tensorflow_amd.train.hooks import CheckpointHook, StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        cluster = ClusterInfo(rank=rank, world=2, device="cuda:0", backend="gloo")
        sess = TrainingSession(cifar_resnet_v2(8), 8, cluster, weight_decay=2e-4,
                               lr_schedule=lr_mod.for_dataset("cifar10"), checkpoint_dir=ck if rank == 0 else "",
                               use_graph=(mode == "stall"), allreduce="p2p", bucket_mb=0.05,
                               step_trial=False)   # (stall: the whole-step graph, no mode trial)
        assert sess.engine.p2p is not None and len(sess.engine.buckets) > 1
        assert sess.use_graph == (mode == "stall")
        feeder = SyntheticFeeder(sess.ex, seed=rank)
        for _ in range(2):
            feeder.next()
            sess.step()
        torch.cuda.synchronize()
        sess.engine.check_errors()
        if rank == 0:
            sess.save(2)
            sess.saver.wait()
        dist.barrier()
        if rank == 1:
            if mode == "withhold":
                sess.engine.p2p.withhold = 0
                sess.step()
                torch.cuda.synchronize()
            q.put((1, "stopped"))
            stop.wait(300)
            os._exit(0)
        w0, m0 = sess.ex.P.master.clone(), sess.ex.P.momentum.clone()
        save_fn = lambda step, blocking: sess.save(step, blocking)  # noqa: E731
        t0 = time.time()
        err = None
        print(f"[rank 0] failing phase starts ({mode})", file=sys.stderr, flush=True)
        try:
            sess.run(feeder, [StopAtStepHook(4)], chief_hooks=[CheckpointHook(0, save_fn)])
        except RuntimeError as e:
            err = str(e)
        dt = time.time() - t0
        print(f"[rank 0] run() returned after {dt:.1f} s: {err}", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        print("[rank 0] device drained", file=sys.stderr, flush=True)
        same = torch.equal(w0, sess.ex.P.master) and torch.equal(m0, sess.ex.P.momentum)
        later = sorted(f for f in os.listdir(ck) if f.startswith("model.ckpt-") and not f.startswith("model.ckpt-2."))
        q.put((0, (err, dt, same, later, sess.failed)))
        _flush(q)
        os._exit(1 if err else 0)
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
        _flush(q)
        os._exit(2)


@pytest.mark.timeout(170)
@pytest.mark.parametrize("mode", ["withhold", "stall"])
def test_p2p_peer_failure_skips_update_and_aborts(tmp_path, mode):
    ctx = mp.get_context("spawn")
    q, stop = ctx.Queue(), ctx.Event()
    port = _free_port()
    ck = str(tmp_path / "ck")
    ps = [ctx.Process(target=_worker, args=(r, mode, port, ck, q, stop)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        while len(res) < 2:
            r, v = q.get(timeout=150)
            res[r] = v
            if isinstance(v, str) and v != "stopped":
                break  # a rank failed outside the injected fault: the other may be stuck in a collective
    finally:
        stop.set()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res.get(1) == "stopped", res
    assert isinstance(res.get(0), tuple), res
    err, dt, same, later, failed = res[0]
    assert err is not None and "P2P all-reduce timed out" in err, res[0]
    assert failed, res[0]
    assert dt < 120, dt                      # a few 1 s device timeouts, not a hang
    assert same, "weights / momentum changed by a step whose exchange failed"
    assert later == [], later                # no checkpoint after the failure
    assert os.path.exists(os.path.join(ck, "model.ckpt-2.index"))
    assert ps[0].exitcode == 1, ps[0].exitcode
