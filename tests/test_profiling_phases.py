"""the training step carries roctx ranges for its phases (data / fwd / bwd / comm /
optimizer) when profiling is on (ProfileHook or DRN_ROCTX=1), and none otherwise."""
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
from distributed_resnet_tensorflow_amd.parallel.cluster import ClusterInfo
from distributed_resnet_tensorflow_amd.train import lr as lr_mod
from distributed_resnet_tensorflow_amd.train.feeder import SyntheticFeeder
from distributed_resnet_tensorflow_amd.train.hooks import StopAtStepHook
from distributed_resnet_tensorflow_amd.train.session import TrainingSession
from distributed_resnet_tensorflow_amd.utils import profiler


class _Rec:
    def __init__(self):
        self.lib = object()
        self.log = []

    def push(self, m):
        self.log.append(("push", m))

    def pop(self):
        self.log.append(("pop", None))


def _run(steps=2):
    sess = TrainingSession(cifar_resnet_v2(8), 2, ClusterInfo(device="cpu"), weight_decay=2e-4,
                           lr_schedule=lr_mod.for_dataset("cifar10"), use_graph=False)
    sess.run(SyntheticFeeder(sess.ex), [StopAtStepHook(steps)])


def test_phase_ranges_when_enabled(monkeypatch):
    rec = _Rec()
    monkeypatch.setattr(profiler, "_ROCTX", rec)
    monkeypatch.setattr(profiler, "_PHASES_ON", True)
    _run(2)
    pushed = [m for k, m in rec.log if k == "push"]
    for name in ("data", "fwd", "bwd", "optimizer"):
        assert pushed.count(name) == 2, (name, pushed)
    assert sum(1 for k, _ in rec.log if k == "pop") == len(pushed)  # balanced


def test_no_ranges_when_disabled(monkeypatch):
    rec = _Rec()
    monkeypatch.setattr(profiler, "_ROCTX", rec)
    monkeypatch.setattr(profiler, "_PHASES_ON", False)
    _run(1)
    assert rec.log == []
