"""End-to-end runs of the reference-named entry points on the CPU (fake CIFAR data):
train -> TF-layout checkpoint -> eval poller -> resume; PS task exit; 2-worker fake cluster;
launcher fault injection + restart-from-checkpoint."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("PYTHONPATH", REPO)
    r = subprocess.run([PY] + args, cwd=REPO, capture_output=True, text=True, timeout=timeout, env=e)
    return r


@pytest.fixture(scope="module")
def cifar_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("cifar")
    sys.path.insert(0, REPO)
    from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar
    write_fake_cifar(str(d), 64)
    return str(d)


def test_single_train_eval_resume(cifar_dir, tmp_path):
    ck, ev = str(tmp_path / "ck"), str(tmp_path / "ev")
    common = [f"--train_data_path={cifar_dir}", f"--log_root={ck}", f"--eval_dir={ev}", "--resnet_size=8",
              "--batch_size=16", "--log_every_n_steps=5", "--save_summaries_steps=5"]
    r = run(["resnet_single.py", "--train_steps=12"] + common)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "step = 10" in r.stdout and os.path.exists(os.path.join(ck, "model.ckpt-12.index"))
    g = open(os.path.join(ck, "graph.pbtxt")).read()   # SURVEY §2.11 artifact (variables-only GraphDef)
    assert 'name: "conv2d/kernel"' in g and 'name: "global_step"' in g and "moving_variance" in g
    r = run(["resnet_cifar_eval.py", "--mode=eval", "--eval_once=True", f"--eval_data_path={cifar_dir}",
             f"--log_root={ck}", f"--eval_dir={ev}", "--resnet_size=8", "--eval_batch_count=2"])
    assert r.returncode == 0 and "precision:" in r.stdout, r.stdout + r.stderr
    assert json.load(open(os.path.join(ev, "best_precision.json")))["step"] == 12
    r = run(["resnet_single.py", "--train_steps=20"] + common)
    assert r.returncode == 0 and "Restored" in r.stdout and "global step 20" in r.stdout, r.stdout + r.stderr


def test_eval_rejects_train_mode(cifar_dir, tmp_path):
    r = run(["resnet_cifar_eval.py", "--mode=train", f"--log_root={tmp_path}"])
    assert r.returncode != 0


def test_ps_task_exits_cleanly(tmp_path):
    r = run(["resnet_cifar_main.py", "--job_name=ps", "--task_index=0", "--ps_hosts=localhost:2230",
             "--worker_hosts=localhost:2220,localhost:2221"])
    assert r.returncode == 0 and "parameter servers are not used" in r.stdout


@pytest.mark.parametrize("shard", [False, True])
def test_two_worker_fake_cluster(cifar_dir, tmp_path, shard):
    """--job_name=worker --task_index=i over localhost ports (reference submit_mac_dist.sh); shard:
    the ZeRO-1 optimizer (--optimizer_sharding), whose checkpoint save is collective."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ck = str(tmp_path / "ck")
    base = ["resnet_cifar_main.py", "--job_name=worker", f"--worker_hosts=127.0.0.1:{port},127.0.0.1:{port + 1}",
            "--ps_hosts=127.0.0.1:2230", "--sync_replicas=True", f"--train_data_path={cifar_dir}", f"--log_root={ck}",
            "--resnet_size=8", "--batch_size=8", "--train_steps=6", "--log_every_n_steps=3"]
    if shard:
        base += ["--optimizer_sharding=True", "--save_checkpoint_secs=1"]
    e = dict(os.environ, PYTHONPATH=REPO)
    ps = [subprocess.Popen([PY] + base + [f"--task_index={i}"], cwd=REPO, env=e, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True) for i in range(2)]
    outs = [p.communicate(timeout=600)[0] for p in ps]
    assert all(p.returncode == 0 for p in ps), outs
    assert "global step 6" in outs[0] and os.path.exists(os.path.join(ck, "model.ckpt-6.index"))
    # SURVEY §5.5 metrics: throughput per node and per GPU, gradient-exchange timing
    import json
    recs = [json.loads(l) for l in open(os.path.join(ck, "metrics.jsonl"))]
    assert recs and all(k in recs[-1] for k in ("images_per_sec", "images_per_sec_per_gpu", "steps_per_sec",
                                                "backward_ms", "comm_exposed_ms"))
    assert abs(recs[-1]["images_per_sec"] - 2 * recs[-1]["images_per_sec_per_gpu"]) < 1e-6 * recs[-1]["images_per_sec"]


def test_launcher_fault_injection_and_restart(cifar_dir, tmp_path):
    ck = str(tmp_path / "ck")
    marker = str(tmp_path / "fault.marker")
    r = run(["-m", "distributed_resnet_tensorflow_amd.parallel.launch", "--nproc", "2", "--max_restarts", "1",
             "resnet_cifar_main_horovod.py", f"--train_data_path={cifar_dir}", f"--log_root={ck}", "--resnet_size=8",
             "--batch_size=8", "--train_steps=8", "--save_checkpoint_secs=0", "--fault_inject_step=5",
             "--fault_inject_rank=1", "--log_every_n_steps=4"],
            env={"DRN_FAULT_MARKER": marker})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert os.path.exists(marker) and "restart 1/1" in r.stderr
    assert os.path.exists(os.path.join(ck, "model.ckpt-8.index"))
