"""Launcher scripts keep the reference's environment interface: the Slurm/local
train+eval launcher and the localhost PS/worker fake cluster (reference
scripts/run_dist_train_eval_daint.sh, scripts/submit_mac_dist.sh), run here on CPU/gloo."""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ, PYTHONPATH=REPO, PYTHON=sys.executable, OMP_NUM_THREADS="2")
    env.update(kw)
    return env


def test_train_eval_launcher_two_ranks_with_sidecar(tmp_path):
    sys.path.insert(0, REPO)
    from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar
    write_fake_cifar(str(tmp_path / "data"), 100)
    env = _env(TF_SCRIPT=os.path.join(REPO, "resnet_cifar_main.py"),
               TF_EVAL_SCRIPT=os.path.join(REPO, "resnet_cifar_eval.py"),
               TF_NUM_PS="1", TF_NUM_WORKERS="2", TF_WORKER_PER_NODE="2", DRN_EVAL_GRACE="8",
               TF_FLAGS=f"--train_data_path={tmp_path}/data --log_root=./ck --dataset=cifar10 --num_gpus=0 "
                        "--batch_size=8 --train_steps=4 --resnet_size=8 --log_every_n_steps=2",
               TF_EVAL_FLAGS=f"--eval_data_path={tmp_path}/data/cifar-10-batches-bin/test_batch* --log_root=./ck "
                             "--eval_dir=./ck/test --dataset=cifar10 --mode=eval --num_gpus=0 "
                             "--eval_batch_count=1 --eval_interval_secs=1 --resnet_size=8")
    r = subprocess.run([os.path.join(REPO, "scripts", "run_dist_train_eval.sh")], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "parameter servers are not used" in r.stdout
    logs = sorted(glob.glob(str(tmp_path / "worker.*.log")))
    assert len(logs) == 2
    assert "training finished at global step 4" in open(logs[0]).read()
    assert (tmp_path / "ck" / "checkpoint").exists()
    assert glob.glob(str(tmp_path / "eval.*.log"))


def test_local_fake_cluster_ps_and_workers(tmp_path):
    env = _env(TF_FLAGS="--synthetic_data=True --log_root=./ck --dataset=cifar10 --num_gpus=0 --batch_size=4 "
                        "--sync_replicas=True --train_steps=3 --resnet_size=8")
    r = subprocess.run([os.path.join(REPO, "scripts", "submit_local_dist.sh"), "1", "2"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "not used by the all-reduce engine" in open(tmp_path / "ps0.log").read()
    for w in ("wk0.log", "wk1.log"):
        assert "training finished at global step 3" in open(tmp_path / w).read()
    assert not (tmp_path / ".drn_pids").read_text().strip() == ""
    k = subprocess.run([os.path.join(REPO, "scripts", "kill.sh")], cwd=tmp_path, env=_env(GRACE="0"),
                       capture_output=True, text=True, timeout=60)
    assert k.returncode == 0 and not (tmp_path / ".drn_pids").exists()
