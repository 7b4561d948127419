import os
import struct

import numpy as np
import pytest
import torch

from distributed_resnet_tensorflow_amd.ckpt import bundle
from distributed_resnet_tensorflow_amd.ckpt.saver import Saver, latest_checkpoint, read_state
from distributed_resnet_tensorflow_amd.utils import crc32c, events, tfrecord


def test_crc32c_known_vectors():
    assert crc32c.value(b"123456789") == 0xE3069283
    assert crc32c.value(b"") == 0
    c = crc32c.value(b"hello world")
    assert crc32c.unmask(crc32c.mask(c)) == c
    # native and python paths agree
    from distributed_resnet_tensorflow_amd.utils import native
    if native.host_lib() is not None:
        data = os.urandom(1000)
        t = crc32c._py_table()
        crc = 0xFFFFFFFF
        for b in data:
            crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
        assert crc32c.value(data) == crc ^ 0xFFFFFFFF


def test_bundle_roundtrip_and_sstable_format(tmp_path):
    rng = np.random.default_rng(0)
    tensors = {f"conv2d_{i}/kernel": rng.standard_normal((3, 3, 4, i + 1)).astype(np.float32) for i in range(40)}
    tensors["global_step"] = np.array(1234, dtype=np.int64)
    tensors["dense/bias"] = np.zeros(10, np.float32)
    prefix = str(tmp_path / "model.ckpt-1234")
    bundle.write_bundle(prefix, tensors)
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == bundle.TABLE_MAGIC
    back = bundle.read_bundle(prefix)
    assert set(back) == set(tensors)
    for k in tensors:
        assert back[k].shape == tensors[k].shape and back[k].dtype == tensors[k].dtype
        np.testing.assert_array_equal(back[k], tensors[k])
    assert back["global_step"].shape == ()
    # corrupted data is detected
    with open(prefix + ".data-00000-of-00001", "r+b") as f:
        f.seek(100)
        f.write(b"\xff\xff\xff\xff")
    with pytest.raises(ValueError):
        bundle.read_bundle(prefix)


def test_saver_rotation_and_state(tmp_path):
    s = Saver(str(tmp_path), max_to_keep=2)
    for step in (10, 20, 30):
        s.save(step, {"w": np.full(3, step, np.float32), "global_step": np.array(step, np.int64)}, blocking=False)
    s.wait()
    st = read_state(str(tmp_path))
    assert st["model_checkpoint_path"] == "model.ckpt-30"
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-20", "model.ckpt-30"]
    assert not os.path.exists(tmp_path / "model.ckpt-10.index")
    p = latest_checkpoint(str(tmp_path))
    assert p.endswith("model.ckpt-30") and int(Saver.restore(p)["global_step"]) == 30


def test_events_roundtrip(tmp_path):
    w = events.EventFileWriter(str(tmp_path))
    w.add_scalars(100, {"Precision": 0.5, "cost": 2.25})
    w.add_scalar("Precision", 0.75, 200)
    w.add_images(200, "images", np.zeros((2, 8, 8, 3), np.uint8), max_images=2)
    w.close()
    assert events.scalar_series(str(tmp_path), "Precision") == [(100, 0.5), (200, 0.75)]
    recs = list(tfrecord.read_records(w.path))
    assert len(recs) == 4  # file_version + 3 events


def test_executor_state_roundtrip(tmp_path):
    from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2
    from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
    from distributed_resnet_tensorflow_amd.runtime.executor import Executor
    from distributed_resnet_tensorflow_amd.runtime.state import export_state, import_state
    spec = cifar_resnet_v2(8)
    a = Executor(spec, 2, RefBackend(), "cpu", seed=1)
    a.P.momentum.normal_()
    a.P.bn_state.uniform_()
    a.P.global_step = 77
    t = export_state(a, {"data_epoch": 3})
    assert t["conv2d/kernel"].shape == (3, 3, 3, 16) and t["dense/kernel"].shape == (64, 10)
    assert "batch_normalization/moving_variance" in t and "conv2d/kernel/Momentum" in t
    bundle.write_bundle(str(tmp_path / "c"), t)
    b = Executor(spec, 2, RefBackend(), "cpu", seed=2)
    extra = import_state(b, bundle.read_bundle(str(tmp_path / "c")))
    assert extra == {"data_epoch": 3} and b.P.global_step == 77
    t2 = export_state(b, {"data_epoch": 3})
    assert set(t2) == set(t)
    for k in t:
        np.testing.assert_array_equal(t[k], t2[k])
