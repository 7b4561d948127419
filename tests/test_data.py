import numpy as np
import torch

from distributed_resnet_tensorflow_amd.data import cifar, imagenet
from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
from distributed_resnet_tensorflow_amd.utils import tfrecord


def test_cifar_records_and_loader(tmp_path):
    cifar.write_fake_cifar(str(tmp_path), 50)
    files = cifar.get_filenames(True, str(tmp_path))
    assert len(files) == 5 and files[0].endswith("data_batch_1.bin")
    rec = cifar.CifarRecords(files)
    assert rec.n == 250
    imgs = np.empty((3, 32, 32, 3), np.uint8)
    labs = np.empty(3, np.int32)
    rec.gather(np.array([0, 7, 249]), imgs, labs)
    raw = np.fromfile(files[0], np.uint8).reshape(50, 3073)
    assert labs[0] == raw[0, 0]
    np.testing.assert_array_equal(imgs[0], raw[0, 1:].reshape(3, 32, 32).transpose(1, 2, 0))
    # rank sharding is disjoint and epoch-deterministic
    l0 = cifar.CifarLoader(rec, 25, True, seed=3, rank=0, world=2)
    l1 = cifar.CifarLoader(rec, 25, True, seed=3, rank=1, world=2)
    p0, p1 = l0._perm(0), l1._perm(0)
    assert len(set(p0.tolist()) & set(p1.tolist())) == 0 and len(p0) == 125
    b = next(l0)
    assert b[0].shape == (25, 32, 32, 3) and b[2].shape == (25, 3) and b[2][:, :2].max() <= 8
    l0.close()
    l1.close()
    # glob pattern form used by the eval scripts (`--eval_data_path=.../test_batch*`)
    assert cifar.get_filenames(False, str(tmp_path / "cifar-10-batches-bin" / "test_batch*"))


def test_cifar100_layout(tmp_path):
    cifar.write_fake_cifar(str(tmp_path), 20, dataset="cifar100")
    rec = cifar.CifarRecords(cifar.get_filenames(True, str(tmp_path), "cifar100"), "cifar100")
    assert rec.record_bytes == 3074 and rec.n == 20
    imgs = np.empty((1, 32, 32, 3), np.uint8)
    labs = np.empty(1, np.int32)
    rec.gather(np.array([0]), imgs, labs)
    raw = np.fromfile(cifar.get_filenames(True, str(tmp_path), "cifar100")[0], np.uint8).reshape(20, 3074)
    assert labs[0] == raw[0, 1]  # fine label (label_offset 1)


def test_cifar_augment_semantics():
    be = RefBackend()
    raw = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    params = torch.tensor([[4, 4, 0], [0, 8, 1]], dtype=torch.int32)
    out = torch.zeros(2, 32, 32, 8)
    be.cifar_augment(raw, params, out, 4)
    x = out[0, :, :, :3]
    assert abs(x.mean().item()) < 1e-4 and abs(x.std(unbiased=False).item() - 1) < 1e-3
    assert out[..., 3:].abs().max() == 0
    # crop (0, 8) flipped: output column 0 = source column (31 - 0) + 8 - 4 -> out of range (zero pad)
    img1 = raw[1].float()
    padded = torch.nn.functional.pad(img1.permute(2, 0, 1), (4, 4, 4, 4))
    crop = padded[:, 0:32, 8:40].flip(2)
    std = (crop - crop.mean()) / crop.std(unbiased=False).clamp_min(1 / np.sqrt(3072))
    assert torch.allclose(out[1, :, :, :3], std.permute(1, 2, 0), atol=1e-4)


def test_imagenet_example_roundtrip_and_vgg(tmp_path):
    paths = imagenet.write_fake_imagenet(str(tmp_path), shards=2, per_shard=3)
    assert imagenet.filenames(True, str(tmp_path)) == paths
    recs = list(tfrecord.read_records(paths[0]))
    assert len(recs) == 3
    ex = imagenet.parse_example(recs[0])
    img = imagenet.decode_image(ex["image/encoded"][0])
    assert img.ndim == 3 and img.shape[2] == 3 and 1 <= ex["image/class/label"][0] <= 1000
    rng = np.random.default_rng(0)
    rh, rw, cy, cx, flip = imagenet.draw_geometry(img.shape[0], img.shape[1], True, rng)
    assert min(rh, rw) >= 256 and 0 <= cy <= rh - 224 and 0 <= cx <= rw - 224
    out = imagenet.vgg_preprocess_np(img, rh, rw, cy, cx, flip)
    assert out.shape == (224, 224, 3)
    # identity geometry reproduces the mean-subtracted pixels
    o2 = imagenet.vgg_preprocess_np(img, img.shape[0], img.shape[1], 0, 0, 0, out=32)
    np.testing.assert_allclose(o2, img[:32, :32] / 255.0 - np.array(imagenet.RGB_MEANS), atol=1e-5)
    rh, rw, cy, cx, flip = imagenet.draw_geometry(300, 400, False, rng)
    assert (rh, rw) == (256, 341) and (cy, cx) == (16, 58) and flip == 0


def test_imagenet_loader_batches(tmp_path):
    imagenet.write_fake_imagenet(str(tmp_path), shards=2, per_shard=4)
    ld = imagenet.ImagenetLoader(str(tmp_path), 3, True, num_threads=2, num_epochs=1)
    packed, desc, labels = next(ld)
    assert desc.shape == (3,) and labels.shape == (3,)
    assert packed.size == int((desc["H"].astype(np.int64) * desc["W"] * 3).sum())
    be = RefBackend()
    out = torch.zeros(3, 224, 224, 8)
    be.vgg_preprocess(packed, desc, out, imagenet.RGB_MEANS)
    assert torch.isfinite(out).all() and out[..., 3:].abs().max() == 0
    ld.close()


def test_imagenet_loader_process_workers_match_threads(tmp_path):
    """Spawned decode processes (pixels through named shared memory) give the same batches as
    the thread pool, and leave no segment behind in /dev/shm."""
    import glob
    import os
    imagenet.write_fake_imagenet(str(tmp_path), shards=2, per_shard=6)
    got = {}
    for w in ("thread", "process"):
        ld = imagenet.ImagenetLoader(str(tmp_path), 4, True, seed=4, num_threads=2, num_epochs=1, workers=w)
        got[w] = [tuple(np.array(x, copy=True) for x in next(ld)) for _ in range(3)]
        ld.close()
    for a, b in zip(got["thread"], got["process"]):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    assert not glob.glob(f"/dev/shm/{imagenet._SHM_PREFIX}{os.getpid()}_*")


def _drain(loader, n):
    out = []
    for _ in range(n):
        b = next(loader)
        out.append(tuple(np.array(x, copy=True) for x in b))
    return out


def test_cifar_loader_resume_is_exact(tmp_path):
    """A loader restarted from the position recorded after batch k yields batch k+1 (same
    images, labels and crop/flip draws), across an epoch boundary too."""
    cifar.write_fake_cifar(str(tmp_path), 20)
    rec = cifar.CifarRecords(cifar.get_filenames(True, str(tmp_path)))
    ld = cifar.CifarLoader(rec, 16, True, seed=5)
    ref, states = [], []
    for _ in range(9):  # 100 records / 16 -> 6 batches per epoch: crosses into epoch 1
        ref.append(tuple(np.array(x, copy=True) for x in next(ld)))
        states.append(ld.state())
    ld.close()
    for k in (0, 4, 5, 7):
        r = cifar.CifarLoader(rec, 16, True, seed=5, epoch=states[k]["data_epoch"], cursor=states[k]["data_cursor"])
        got = _drain(r, 1)[0]
        r.close()
        for a, b in zip(got, ref[k + 1]):
            np.testing.assert_array_equal(a, b)


def test_cifar_eval_partial_batch_valid_count(tmp_path):
    cifar.write_fake_cifar(str(tmp_path), 50)
    rec = cifar.CifarRecords(cifar.get_filenames(False, str(tmp_path)))
    ld = cifar.CifarLoader(rec, 20, False)
    valids = []
    for _ in range(3):
        next(ld)
        valids.append(ld.valid)
    ld.close()
    assert valids == [20, 20, 10]  # the wrapped tail of the last batch is not counted


def test_cifar_feeder_state_is_consumed_batch(tmp_path):
    """CPU feeder: state() after next() is the position after the batch now in the executor
    (not after the prefetched one), and the labels in the executor are that batch's."""
    from distributed_resnet_tensorflow_amd.models.spec import build_spec
    from distributed_resnet_tensorflow_amd.runtime.executor import Executor
    from distributed_resnet_tensorflow_amd.train.feeder import CifarFeeder
    cifar.write_fake_cifar(str(tmp_path), 20)
    rec = cifar.CifarRecords(cifar.get_filenames(True, str(tmp_path)))
    ref_ld = cifar.CifarLoader(rec, 8, True, seed=2)
    ref = _drain(ref_ld, 4)
    ref_ld.close()
    ex = Executor(build_spec("cifar10", 8), 8, RefBackend(), "cpu")
    f = CifarFeeder(ex, cifar.CifarLoader(rec, 8, True, seed=2), True)
    for k in range(4):
        assert f.next()
        np.testing.assert_array_equal(ex.labels.numpy(), ref[k][1])
        assert f.state() == {"data_epoch": 0, "data_cursor": 8 * (k + 1)}
    f.close()


def test_imagenet_loader_resume_is_exact(tmp_path):
    """(epoch, records consumed, batch index) is a complete position: a restarted loader
    continues with the same records and the same crop/flip draws, across epochs."""
    imagenet.write_fake_imagenet(str(tmp_path), shards=3, per_shard=4)
    ld = imagenet.ImagenetLoader(str(tmp_path), 5, True, seed=1, num_threads=2)
    ref, states = [], []
    for _ in range(5):  # 12 records / epoch, 5 per batch: batches straddle epochs
        p, d, l = next(ld)
        ref.append((np.array(p, copy=True), d.copy(), l.copy()))
        states.append(ld.state())
    ld.close()
    assert states[1]["data_epoch"] == 0 and states[2]["data_epoch"] == 1
    for k in (0, 1, 2, 3):
        st = states[k]
        r = imagenet.ImagenetLoader(str(tmp_path), 5, True, seed=1, num_threads=2, epoch=st["data_epoch"],
                                    cursor=st["data_cursor"], batch_index=st["data_batch"])
        p, d, l = next(r)
        r.close()
        np.testing.assert_array_equal(l, ref[k + 1][2])
        np.testing.assert_array_equal(d, ref[k + 1][1])
        np.testing.assert_array_equal(np.asarray(p), ref[k + 1][0])


def test_imagenet_epoch_order_is_a_permutation(tmp_path):
    imagenet.write_fake_imagenet(str(tmp_path), shards=3, per_shard=7)
    ld = imagenet.ImagenetLoader(str(tmp_path), 4, True, seed=3, num_threads=1, num_epochs=1)
    o0, o1 = list(ld.epoch_order(0)), list(ld.epoch_order(1))
    ld.close()
    assert sorted(o0) == sorted(o1) == [(s, r) for s in range(3) for r in range(7)]
    assert o0 != o1
