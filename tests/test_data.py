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
