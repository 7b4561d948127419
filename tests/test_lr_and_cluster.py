from distributed_resnet_tensorflow_amd import flags
from distributed_resnet_tensorflow_amd.parallel.cluster import resolve
from distributed_resnet_tensorflow_amd.train import lr


def test_cifar_schedule_boundaries():
    assert lr.cifar_lr(0) == 0.1 and lr.cifar_lr(39999) == 0.1 and lr.cifar_lr(40000) == 0.01
    assert lr.cifar_lr(59999) == 0.01 and lr.cifar_lr(60000) == 0.001
    assert lr.cifar_lr(79999) == 0.001 and lr.cifar_lr(80000) == 0.0001


def test_imagenet_schedule_boundaries():
    assert abs(lr.imagenet_lr(0) - 0.1) < 1e-12
    assert abs(lr.imagenet_lr(3120) - 0.25) < 1e-12
    assert lr.imagenet_lr(6239) < 0.4 and lr.imagenet_lr(6240) == 0.4
    assert lr.imagenet_lr(37439) == 0.4 and lr.imagenet_lr(37440) == 0.04
    assert lr.imagenet_lr(74880) == 0.004 and lr.imagenet_lr(99840) == 0.0004


def test_first_step_uses_begin_value():
    s = lr.for_dataset("imagenet")
    assert s.lr_for_step() == 0.4  # reference begin() quirk, resnet_imagenet_main.py:226-227
    s.after_step(0)
    assert abs(s.lr_for_step() - 0.1) < 1e-12


def _fv(*args):
    fv = flags.FlagValues()
    flags.define_reference_flags(fv)
    fv(["p"] + list(args))
    return fv


def test_cluster_ps_worker_mapping():
    fv = _fv("--job_name=worker", "--task_index=2", "--worker_hosts=h0:2220,h1:2221,h2:2222", "--ps_hosts=p:2230")
    c = resolve(fv, env={})
    assert (c.rank, c.world, c.master_addr, c.master_port) == (2, 3, "h0", 2220)
    assert not c.is_chief and c.backend == "gloo"
    assert resolve(_fv("--job_name=ps", "--task_index=0"), env={}).role == "ps"


def test_cluster_env_and_mpi():
    c = resolve(_fv(), env={"WORLD_SIZE": "4", "RANK": "1", "LOCAL_RANK": "1", "MASTER_ADDR": "10.0.0.1",
                            "MASTER_PORT": "1234"})
    assert (c.rank, c.world, c.local_rank, c.master_port) == (1, 4, 1, 1234)
    c = resolve(_fv(), env={"OMPI_COMM_WORLD_SIZE": "2", "OMPI_COMM_WORLD_RANK": "0"})
    assert c.world == 2 and c.is_chief
    assert resolve(_fv(), env={}).role == "serial"
