"""End-to-end runs of the reference-named entry points on the GPU (HIP kernels, HIP-graph step):

  * resnet_cifar_main.py --num_gpus=1 on a class-conditional fake CIFAR-10 (learnable: one hue
    per class) with the reference LR schedule compressed 20x (--lr_schedule_scale=0.05: 0.1,
    0.01 from step 2000, 0.001 from 3000) -> checkpoint -> resnet_cifar_eval.py --eval_once=True
    must report held-out precision >= 0.95 and >= 0.98 on the training records -- convergence
    of the whole GPU train + eval path (accuracy parity with the reference's 93 % on real
    CIFAR-10 is unpinned: no dataset here);
  * resnet_imagenet_main.py / resnet_imagenet_eval.py on fake TFRecord shards (default model =
    ResNet-v2-50) -> checkpoint -> eval.
"""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def run(args, timeout=280):
    e = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([PY, "-u"] + args, cwd=REPO, capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, (args[0], r.stdout[-4000:], r.stderr[-4000:])
    return r.stdout + r.stderr


@pytest.mark.timeout(600)
def test_cifar_gpu_train_checkpoint_eval_converges(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar
    data = str(tmp_path / "data")
    write_fake_cifar(data, 1000, learnable=True)
    ck, ev = str(tmp_path / "ck"), str(tmp_path / "ev")
    out = run(["resnet_cifar_main.py", "--num_gpus=1", f"--train_data_path={data}", f"--log_root={ck}",
               "--resnet_size=8", "--batch_size=128", "--train_steps=3000", "--lr_schedule_scale=0.05",
               "--log_every_n_steps=50"])
    assert "global step 3000" in out, out[-2000:]
    assert os.path.exists(os.path.join(ck, "model.ckpt-3000.index"))
    train_prec = [float(v) for v in re.findall(r"precision = ([0-9.]+)", out)]
    assert train_prec and max(train_prec[-5:]) >= 0.95, out[-2000:]
    # Eval normalises with the BN MOVING statistics (decay 0.997, reference
    # resnet_model_official.py:37). Root cause of the round-2 spread (0.67-1.0 held out, the SAME
    # on the training records, batch-statistics precision 1.0: scripts/probes/cifar_eval_probe.sh,
    # profiles/r3_cifar_eval_probe.txt): at a constant LR of 0.1 the weights keep moving faster
    # than a 0.997 average (~330-step horizon) can follow; the reference only evaluates after its
    # 40k/60k-step decays. With the compressed schedule the averages catch up.
    for name, pattern, bar in (("test", "test_batch*", 0.95), ("train", "data_batch_*", 0.98)):
        out = run(["resnet_cifar_eval.py", "--mode=eval", "--eval_once=True", "--num_gpus=1",
                   f"--eval_data_path={data}/cifar-10-batches-bin/{pattern}", f"--log_root={ck}",
                   f"--eval_dir={ev}_{name}", "--resnet_size=8", "--eval_batch_count=10"])
        m = re.findall(r"precision: ([0-9.]+), best precision", out)
        assert m, out[-2000:]
        assert float(m[-1]) >= bar, (name, out[-2000:])
    best = json.load(open(os.path.join(ev + "_test", "best_precision.json")))
    assert best["step"] == 3000 and best["best_precision"] >= 0.95


@pytest.mark.timeout(600)
def test_imagenet_gpu_train_checkpoint_eval(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_resnet_tensorflow_amd.data.imagenet import write_fake_imagenet
    data = str(tmp_path / "data")
    write_fake_imagenet(data, shards=2, per_shard=8, is_training=True)
    write_fake_imagenet(data, shards=1, per_shard=8, is_training=False, seed=1)
    ck, ev = str(tmp_path / "ck"), str(tmp_path / "ev")
    out = run(["resnet_imagenet_main.py", "--num_gpus=1", f"--train_data_path={data}", f"--log_root={ck}",
               "--batch_size=4", "--train_steps=6", "--log_every_n_steps=2"])
    assert "global step 6" in out, out[-2000:]
    from distributed_resnet_tensorflow_amd.ckpt.saver import Saver, latest_checkpoint
    t = Saver.restore(latest_checkpoint(ck))
    assert t["conv2d/kernel"].shape == (7, 7, 3, 64)
    n = sum(int(v.size) for k, v in t.items() if not k.endswith("Momentum") and "moving" not in k
            and k != "global_step" and not k.startswith("drn/"))
    assert n == 25_551_401  # ResNet-v2-50 by default (not the WRN-50-2 of round 1)
    assert "drn/data_cursor" in t and "drn/data_batch" in t  # input-pipeline position for resume
    out = run(["resnet_imagenet_eval.py", "--mode=eval", "--eval_once=True", "--num_gpus=1",
               f"--eval_data_path={data}", f"--log_root={ck}", f"--eval_dir={ev}", "--batch_size=4",
               "--eval_batch_count=2"])
    assert re.search(r"precision: [0-9.]+, best precision", out), out[-2000:]
