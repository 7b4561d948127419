"""GPU checks of the evaluation path and the input pipelines:

  * inference-mode forward (BN moving statistics restored from a checkpoint) vs the fp32
    autograd oracle, CIFAR and ImageNet ResNet-50;
  * the fused VGG resize/crop/flip/mean kernel (drn_vgg_preprocess) vs its numpy mirror;
  * the CIFAR and ImageNet GPU feeders with the host running far ahead of the GPU: every
    batch that reaches the executor is the loader's batch, in order;
  * ImageNet feeder resume: a loader restarted from the checkpointed position continues with
    the next unconsumed batch.
"""
import numpy as np
import pytest
import torch

from distributed_resnet_tensorflow_amd.data import cifar, imagenet
from distributed_resnet_tensorflow_amd.models import oracle
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2, imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend, RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor
from distributed_resnet_tensorflow_amd.runtime.state import export_state, import_state
from distributed_resnet_tensorflow_amd.train.feeder import CifarFeeder, ImagenetFeeder

pytestmark = pytest.mark.gpu


def _busy(n=6):
    """~10 ms of GPU work on the current stream: the host runs ahead while it executes."""
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(n):
        a = torch.tanh(a @ a * 1e-3)
    return a


@pytest.mark.parametrize("which", ["cifar20", "in50"])
def test_eval_forward_matches_oracle(which):
    spec, N = {"cifar20": (cifar_resnet_v2(20), 32), "in50": (imagenet_resnet_v2(50), 4)}[which]
    g = torch.Generator().manual_seed(11)
    S = spec.image_size
    # a few training steps on HIP so the moving statistics are far from their (0, 1) init
    tr = Executor(spec, N, HipBackend(), "cuda", seed=4)
    for _ in range(3):
        tr.images.zero_()
        tr.images[..., :3] = (torch.randn(N, S, S, 3, generator=g) * 1.5 + 0.2).bfloat16().cuda()
        tr.labels.copy_(torch.randint(0, spec.num_classes, (N,), generator=g, dtype=torch.int32))
        tr.train_step(lr=0.02)
    torch.cuda.synchronize()
    ck = export_state(tr)
    # fresh executor restored from the checkpoint tensors (what the eval poller does)
    ev = Executor(spec, N, HipBackend(), "cuda", seed=99)
    import_state(ev, ck)
    imgs = (torch.randn(N, S, S, 3, generator=g) * 1.5 + 0.2).bfloat16()
    labels = torch.randint(0, spec.num_classes, (N,), generator=g, dtype=torch.int32)
    ev.images.zero_()
    ev.images[..., :3] = imgs.cuda()
    ev.labels.copy_(labels.cuda())
    ev.forward(train=False)
    torch.cuda.synchronize()
    # oracle on the same bf16-rounded weights (the HIP path computes with bf16 weight copies)
    p = {s.name: torch.from_numpy(ck[s.name]).bfloat16().float() for s in tr.P.slots}
    st = {bn: (torch.from_numpy(ck[f"{bn}/moving_mean"]), torch.from_numpy(ck[f"{bn}/moving_variance"]))
          for bn in tr.P.bn_slots}
    mv_before = {k: (a.clone(), b.clone()) for k, (a, b) in st.items()}
    with torch.no_grad():
        logits = oracle.forward(spec, p, st, imgs.float(), training=False)
    for k in st:  # inference must not touch the moving statistics
        assert torch.equal(st[k][0], mv_before[k][0]) and torch.equal(st[k][1], mv_before[k][1])
    h = ev.logits.float().cpu()
    cos = torch.nn.functional.cosine_similarity(h.flatten(), logits.flatten(), dim=0).item()
    assert cos > 0.99, cos
    xent = torch.nn.functional.cross_entropy(logits, labels.long(), reduction="none")
    assert torch.allclose(ev.loss_vec.cpu(), xent, atol=0.05 + 0.02 * xent.abs().max().item())
    # the eval step did not move the executor's moving statistics either
    for bn in ev.P.bn_slots:
        m, v = ev.P.moving(bn)
        assert torch.allclose(m.float().cpu(), mv_before[bn][0]) and torch.allclose(v.float().cpu(), mv_before[bn][1])


def test_vgg_preprocess_kernel_matches_numpy():
    rng = np.random.default_rng(3)
    imgs, descs = [], []
    off = 0
    cases = [(240, 320, True), (333, 250, True), (256, 256, False), (500, 375, True), (231, 600, False),
             (300, 300, True), (224, 224, False), (410, 260, True)]
    for i, (H, W, train) in enumerate(cases):
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        rh, rw, cy, cx, flip = imagenet.draw_geometry(H, W, train, rng)
        if train:
            flip = i % 2  # both flip states for sure
        descs.append((off, H, W, rh, rw, cy, cx, flip, 0))
        imgs.append(img)
        off += img.size
    packed = np.concatenate([x.reshape(-1) for x in imgs])
    desc = np.array(descs, dtype=imagenet.IMG_DESC)
    out = torch.zeros(len(cases), 224, 224, 8, dtype=torch.bfloat16, device="cuda")
    HipBackend().vgg_preprocess(torch.from_numpy(packed).cuda(), torch.from_numpy(desc.view(np.uint8)).cuda(), out,
                                imagenet.RGB_MEANS)
    torch.cuda.synchronize()
    o = out.float().cpu().numpy()
    assert np.all(o[..., 3:] == 0)
    for i, (img, d) in enumerate(zip(imgs, descs)):
        ref = imagenet.vgg_preprocess_np(img, *d[3:8])
        err = np.abs(o[i, :, :, :3] - ref).max()
        assert err <= 1.0 / 255, (i, d, err)


def test_cifar_feeder_host_ahead_keeps_batches(tmp_path):
    cifar.write_fake_cifar(str(tmp_path), 120)
    rec = cifar.CifarRecords(cifar.get_filenames(True, str(tmp_path)))
    N, steps = 64, 24   # 600 records / 64 -> 9 batches an epoch: crosses two epoch boundaries
    ref_ld = cifar.CifarLoader(rec, N, True, seed=4)
    ref = [tuple(np.array(x, copy=True) for x in next(ref_ld)) for _ in range(steps)]
    ref_ld.close()
    ex = Executor(cifar_resnet_v2(8), N, HipBackend(), "cuda")
    f = CifarFeeder(ex, cifar.CifarLoader(rec, N, True, seed=4, pin=True, pin_device=ex.device), True)
    hist_lab = torch.empty(steps, N, dtype=torch.int32, device="cuda")
    hist_img = torch.empty(steps, N, 32, 32, 3, dtype=torch.bfloat16, device="cuda")
    for k in range(steps):
        assert f.next()
        # what the step consumes: the augmented batch in the executor's input buffers
        hist_lab[k].copy_(ex.labels)
        hist_img[k].copy_(ex.images[..., :3])
        _busy()   # the host enqueues the next prefetches long before this finishes
    torch.cuda.synchronize()
    f.close()
    rb = RefBackend()
    for k in range(steps):
        np.testing.assert_array_equal(hist_lab[k].cpu().numpy(), ref[k][1], err_msg=f"labels of batch {k}")
        want = torch.zeros(N, 32, 32, 8)
        rb.cifar_augment(torch.from_numpy(ref[k][0]), torch.from_numpy(ref[k][2]), want, cifar.PAD)
        err = (hist_img[k].float().cpu() - want[..., :3]).abs().max().item()
        assert err < 0.03, (k, err)  # bf16 rounding of standardised pixels; a wrong batch is O(1)


def test_imagenet_feeder_gpu_vs_cpu_and_resume(tmp_path):
    imagenet.write_fake_imagenet(str(tmp_path), shards=3, per_shard=6)
    spec = imagenet_resnet_v2(18)
    N, steps = 4, 6

    def loader(pin, **kw):
        return imagenet.ImagenetLoader(str(tmp_path), N, True, seed=2, num_threads=2, pin=pin,
                                       pin_device=torch.device("cuda") if pin else None, **kw)

    cpu = Executor(spec, N, RefBackend(), "cpu")
    fc = ImagenetFeeder(cpu, loader(False), True)
    ref_img, ref_lab, states = [], [], []
    for _ in range(steps):
        assert fc.next()
        ref_img.append(cpu.images[..., :3].clone())
        ref_lab.append(cpu.labels.clone())
        states.append(fc.state())
    fc.close()
    gx = Executor(spec, N, HipBackend(), "cuda")
    fg = ImagenetFeeder(gx, loader(True), True)
    hist_img = torch.empty(steps, N, 224, 224, 3, dtype=torch.bfloat16, device="cuda")
    hist_lab = torch.empty(steps, N, dtype=torch.int32, device="cuda")
    for k in range(steps):
        assert fg.next()
        assert fg.state() == states[k]
        hist_img[k].copy_(gx.images[..., :3])
        hist_lab[k].copy_(gx.labels)
        _busy()
    torch.cuda.synchronize()
    fg.close()
    for k in range(steps):
        assert torch.equal(hist_lab[k].cpu(), ref_lab[k]), k
        err = (hist_img[k].float().cpu() - ref_img[k]).abs().max().item()
        assert err <= 1.0 / 255, (k, err)
    # resume from the position checkpointed after step 2 -> step 3's batch
    st = states[2]
    fr = ImagenetFeeder(gx, loader(True, epoch=st["data_epoch"], cursor=st["data_cursor"],
                                   batch_index=st["data_batch"]), True)
    assert fr.next()
    torch.cuda.synchronize()
    assert torch.equal(gx.labels.cpu(), ref_lab[3])
    assert (gx.images[..., :3].float().cpu() - ref_img[3]).abs().max().item() <= 1.0 / 255
    fr.close()
