"""Topology unit tests (SURVEY §4.2 tier 'Unit: topology'): layer / BN / variable counts,
parameter counts, TF variable naming and creation order, FLOP report,
output shapes of the autograd oracle, and the debug modes of the executor."""
import pytest
import torch

from distributed_resnet_tensorflow_amd.models import oracle
from distributed_resnet_tensorflow_amd.models.spec import build_spec, cifar_resnet_v2, imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor


def _counts(spec):
    convs = 1 + sum(len(b.convs) + (b.proj is not None) for b in spec.blocks)
    bns = sum(1 + len(b.bns) for b in spec.blocks) + 1
    return convs, bns, len(spec.trainable_variables())


def test_appendix_a_counts():
    # CIFAR ResNet-50 (6n+2, n=8): 52 convs, 49 BNs, 152 trainable tensors, 758,618 params
    assert _counts(cifar_resnet_v2(50)) == (52, 49, 152)
    assert cifar_resnet_v2(50).num_params() == 758_618
    # ImageNet ResNet-v2-50, 1001 classes: 53 convs, 49 BNs, 153 tensors, 25,551,401 params
    assert _counts(imagenet_resnet_v2(50)) == (53, 49, 153)
    assert imagenet_resnet_v2(50).num_params() == 25_551_401


@pytest.mark.parametrize("size,params", [(18, 11_689_512), (34, 21_797_672), (101, 44_549_160),
                                         (152, 60_192_808)])
def test_imagenet_family_param_counts(size, params):
    # sanity bound against the well-known v1 / 1000-class counts: the v2 pre-activation layout
    # (BN placement) and the 1001st class change the totals by well under 1 %
    n = imagenet_resnet_v2(size).num_params()
    assert abs(n - params) / params < 0.01, (size, n)


def test_wide_resnet_and_cifar100():
    assert build_spec("imagenet", 50, width=2).num_params() == 68_877_609  # WRN-50-2 (1001 cls)
    s = build_spec("cifar100", 20)
    assert s.num_classes == 100 and _counts(s)[0] == 20 + 2  # 6n+2 convs + 2 projections


def test_cifar_sizes_require_6n_plus_2():
    with pytest.raises(Exception):
        cifar_resnet_v2(21)


def test_tf_variable_names_in_creation_order():
    names = [v[0] for v in cifar_resnet_v2(8).trainable_variables()]
    assert names[0] == "conv2d/kernel"
    assert names[1:3] == ["batch_normalization/gamma", "batch_normalization/beta"]
    assert names[-2:] == ["dense/kernel", "dense/bias"]
    assert len(names) == len(set(names))


def test_flop_report_matches_appendix():
    s = imagenet_resnet_v2(50)
    gf = s.flops() / 1e9 if hasattr(s, "flops") else None
    if gf is not None:
        assert 7.5 < gf < 8.5  # 8.18 GFLOP/img forward (Appendix A)


def test_oracle_output_shapes():
    spec = imagenet_resnet_v2(18, num_classes=10, image_size=64)
    ex = Executor(spec, 2, RefBackend(), "cpu", seed=0)
    p = oracle.params_from_store(ex.P, requires_grad=False)
    st = oracle.state_from_store(ex.P)
    logits, xent, _ = oracle.loss_fn(spec, p, st, ex.images, torch.zeros(2, dtype=torch.long))
    assert logits.shape == (2, 10) and torch.isfinite(xent)


def test_check_nan_mode_names_the_failing_stage(monkeypatch):
    monkeypatch.setenv("DRN_CHECK_NAN", "1")
    spec = cifar_resnet_v2(8)
    ex = Executor(spec, 2, RefBackend(), "cpu", seed=0)
    ex.images.zero_()
    ex.images[0, 0, 0, 0] = float("nan")
    with pytest.raises(FloatingPointError, match="block"):
        ex.train_step(lr=0.1)


def test_deterministic_mode_plans_one_slot_per_workgroup(monkeypatch):
    monkeypatch.setenv("DRN_DETERMINISTIC", "1")
    ex = Executor(cifar_resnet_v2(8), 4, RefBackend(), "cpu", seed=0)
    assert ex.deterministic and not ex.fuse_bn_bwd
    assert all(b.G >= 1024 for bp in ex.blocks for b in bp.bn[1:])
    ex.train_step(lr=0.1)
    assert torch.isfinite(ex.loss_vec).all()
