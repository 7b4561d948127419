"""Single-GPU TrainingSession: the graph step's side-stream trial (train/session.py).

The first replays of the captured step are timed with the weight-gradient side stream, the
step is then re-captured on one stream and timed the same way, and the faster graph is kept;
every replay is a real training step, so training continues without a gap and the global step
counts every one of them."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")]


@pytest.mark.parametrize("trial", ["1", "0"])
def test_graph_step_side_stream_trial(monkeypatch, trial):
    monkeypatch.setenv("DRN_SIDE_TRIAL", trial)
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.feeder import SyntheticFeeder
    from distributed_resnet_tensorflow_amd.train.hooks import StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    sess = TrainingSession(cifar_resnet_v2(8), 16, ClusterInfo(device="cuda:0"), weight_decay=2e-4,
                           lr_schedule=lr_mod.for_dataset("cifar10"), use_graph=True, step_trial=False)
    assert sess.use_graph and sess.engine is None and sess.ex.side is not None
    sess.run(SyntheticFeeder(sess.ex, seed=0), [StopAtStepHook(50)])
    torch.cuda.synchronize()
    assert sess.global_step == 50
    loss = float(sess.ex.metrics()["cross_entropy"])
    assert loss == loss
    if trial == "1":
        c = sess.side_choice
        assert c is not None and c["side_ms"] > 0 and c["one_stream_ms"] > 0, c
        assert (sess.ex.side is None) == (c["mode"] == "one stream")
    else:
        assert sess.side_choice is None and sess.ex.side is not None


def test_p2p_dp_session_step_mode_and_side_stream_trials(monkeypatch):
    """The data-parallel step with the P2P all-reduce (single-rank engine): its first steps time
    the whole-step graph (reductions included) against the native plans with the P2P kernels
    recorded (runtime/plan.py; with and without the side stream) and keep the fastest; a kept
    graph continues with its side-stream trial. Every candidate trains, the global step counts
    every real step, the P2P error word stays clear."""
    monkeypatch.setenv("DRN_SIDE_TRIAL", "1")
    monkeypatch.setenv("DRN_FORCE_DP", "1")
    monkeypatch.setenv("DRN_FORCE_DP_PORT", "29611")
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.feeder import SyntheticFeeder
    from distributed_resnet_tensorflow_amd.train.hooks import StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    import torch.distributed as dist
    try:
        sess = TrainingSession(cifar_resnet_v2(8), 16, ClusterInfo(device="cuda:0"), weight_decay=2e-4,
                               lr_schedule=lr_mod.for_dataset("cifar10"), use_graph=True, allreduce="p2p")
        assert not sess.use_graph and sess._trial is not None
        assert sess.engine is not None and sess.engine.p2p is not None
        sess.run(SyntheticFeeder(sess.ex, seed=0), [StopAtStepHook(100)])
        torch.cuda.synchronize()
        assert sess.global_step == 100 and sess.failed is None   # (run() polled the error word every step)
        c = sess.graph_choice
        assert c is not None and c["graph_ms"] > 0 and c["plan_ms"] > 0 and c["plan_one_stream_ms"] > 0, c
        if c["mode"] == "graph":
            assert sess.use_graph and sess._plan is None
            s = sess.side_choice
            assert s is not None and s["side_ms"] > 0 and s["one_stream_ms"] > 0, s
        else:
            assert c["mode"] in ("native plan", "native plan (one stream)"), c
            assert not sess.use_graph and sess._plan is not None and sess._plan.p2p is not None
        assert float(sess.ex.metrics()["cross_entropy"]) == float(sess.ex.metrics()["cross_entropy"])
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_graph_step_staged_feeder_async_prefetch(tmp_path):
    """The real CIFAR input path under graph steps: staged feeder (pinned loader, H2D copies on
    the feeder's stream), the host prefetch of batch k+1 on the session's worker thread while
    step k is enqueued -- except around the steps that capture a graph (the first step and the
    side-stream trial's re-capture: TrainingSession.will_capture) -- and every step consumes
    the loader's batches in order (feeder prefetch vs graph capture)."""
    import numpy as np
    from distributed_resnet_tensorflow_amd.data import cifar
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.feeder import CifarFeeder
    from distributed_resnet_tensorflow_amd.train.hooks import Hook, StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    cifar.write_fake_cifar(str(tmp_path), 120)
    rec = cifar.CifarRecords(cifar.get_filenames(True, str(tmp_path)))
    N, steps = 32, 40
    ref_ld = cifar.CifarLoader(rec, N, True, seed=7)
    ref = [np.array(next(ref_ld)[1], copy=True) for _ in range(steps)]
    ref_ld.close()
    sess = TrainingSession(cifar_resnet_v2(8), N, ClusterInfo(device="cuda:0"), weight_decay=2e-4,
                           lr_schedule=lr_mod.for_dataset("cifar10"), use_graph=True, step_trial=False)
    captures = []
    hist = torch.empty(steps, N, dtype=torch.int32, device="cuda")

    class Record(Hook):
        def before_step(self, s, step):
            captures.append(s.will_capture())

        def after_step(self, s, step, metrics):
            hist[step - 1].copy_(s.ex.labels)

    feeder = CifarFeeder(sess.ex, cifar.CifarLoader(rec, N, True, seed=7, pin=True, pin_device=sess.ex.device), True)
    sess.run(feeder, [StopAtStepHook(steps), Record()])
    feeder.close()
    torch.cuda.synchronize()
    assert sess.global_step == steps and sess.failed is None
    assert captures[0] and sum(captures) >= 2, captures   # first capture + the trial's re-capture
    for k in range(steps):
        np.testing.assert_array_equal(hist[k].cpu().numpy(), ref[k], err_msg=f"labels of step {k}")
    assert float(sess.ex.metrics()["cross_entropy"]) == float(sess.ex.metrics()["cross_entropy"])


def test_single_gpu_session_times_graph_and_plan():
    """Single-GPU session (no engine): its first steps time the whole-step graph, the native
    plan (runtime/plan.py, one host thread per stream) and the plan recorded on one stream, and
    keep the fastest -- real training steps throughout; a kept graph continues with its
    side-stream trial."""
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
    from distributed_resnet_tensorflow_amd.train import lr as lr_mod
    from distributed_resnet_tensorflow_amd.train.feeder import SyntheticFeeder
    from distributed_resnet_tensorflow_amd.train.hooks import StopAtStepHook
    from distributed_resnet_tensorflow_amd.train.session import TrainingSession
    sess = TrainingSession(cifar_resnet_v2(8), 16, ClusterInfo(device="cuda:0"), weight_decay=2e-4,
                           lr_schedule=lr_mod.for_dataset("cifar10"), use_graph=True)
    assert not sess.use_graph and sess._trial is not None and sess.engine is None
    sess.run(SyntheticFeeder(sess.ex, seed=0), [StopAtStepHook(60)])  # (trial: 3 x 14 steps)
    torch.cuda.synchronize()
    assert sess.global_step == 60 and sess.failed is None
    c = sess.graph_choice
    assert c is not None and c["graph_ms"] > 0 and c["plan_ms"] > 0, c
    assert c["plan_one_stream_ms"] > 0, c
    assert c["mode"] in ("graph", "native plan", "native plan (one stream)"), c
    if c["mode"] == "graph":
        assert sess.use_graph and sess._plan is None
    elif c["mode"] == "native plan":
        assert not sess.use_graph and sess._plan is not None and sess._plan.threads == 2
    else:
        assert not sess.use_graph and sess._plan is not None and sess.ex.side is None
    loss = float(sess.ex.metrics()["cross_entropy"])
    assert loss == loss
