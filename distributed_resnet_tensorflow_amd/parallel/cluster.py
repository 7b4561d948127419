"""Cluster bootstrap: maps the reference's PS/worker CLI and Horovod/MPI/Slurm/torchrun
environments onto one-process-per-GPU torch.distributed ranks.

Reference (resnet_cifar_main.py:350-399): `--job_name={ps,worker} --task_index=i
--ps_hosts=.. --worker_hosts=..` builds a tf.train.ClusterSpec, PS tasks block in
server.join(), worker i uses GPU i % num_gpus, the chief is task 0, and
replicas_to_aggregate = len(worker_hosts). Horovod: hvd.init()/rank()/local_rank() under
mpirun/srun (resnet_cifar_main_horovod.py:122-123, :342).

Here:
  * torchrun / drn launch env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT) wins;
  * `--job_name=worker`: rank = task_index, world = len(worker_hosts), rendezvous at
    worker_hosts[0] (its host:port), GPU = task_index % num_gpus (reference pinning);
  * `--job_name=ps`: there are no parameter servers in an all-reduce engine -> role "ps"; the
    entry point logs a notice and exits 0 (so unchanged launch scripts still work);
  * MPI / Slurm (`mpirun`, `srun` for the Horovod scripts): OMPI_COMM_WORLD_* / PMI_* /
    SLURM_PROCID+SLURM_NTASKS+SLURM_LOCALID, rendezvous at MASTER_ADDR or the first Slurm node;
  * otherwise a single process (the reference "serial" mode).
Backend: "nccl" (= RCCL over xGMI) with GPUs, "gloo" on CPU (--num_gpus=0 or no GPU).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from datetime import timedelta
from typing import Optional

log = logging.getLogger("drn")


@dataclass
class ClusterInfo:
    role: str = "worker"         # worker | ps | serial
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    device: str = "cpu"
    backend: str = "gloo"

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


def _split_host(hp: str):
    hp = hp.strip()
    if ":" in hp:
        h, p = hp.rsplit(":", 1)
        return h, int(p)
    return hp, 29500


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover
        return False


def resolve(flags, env: Optional[dict] = None) -> ClusterInfo:
    env = dict(os.environ if env is None else env)
    want_gpu = (getattr(flags, "num_gpus", 0) or 0) > 0
    gpu = want_gpu and _gpu_available()
    info = ClusterInfo()
    job = getattr(flags, "job_name", None)
    if job == "ps":
        info.role = "ps"
        return info
    if "WORLD_SIZE" in env and "RANK" in env:
        info.world = int(env["WORLD_SIZE"])
        info.rank = int(env["RANK"])
        info.local_rank = int(env.get("LOCAL_RANK", "0"))
        info.master_addr = env.get("MASTER_ADDR", "127.0.0.1")
        info.master_port = int(env.get("MASTER_PORT", "29500"))
    elif job == "worker":
        if flags.task_index is None:
            raise ValueError("Must specify an explicit `task_index`")
        workers = [w for w in flags.worker_hosts.split(",") if w]
        info.world = len(workers)
        info.rank = int(flags.task_index)
        h, p = _split_host(workers[0])
        info.master_addr = flags.master_addr or h
        info.master_port = p
        ng = max(1, flags.num_gpus or 1)
        info.local_rank = info.rank % ng
    elif "OMPI_COMM_WORLD_SIZE" in env:
        info.world = int(env["OMPI_COMM_WORLD_SIZE"])
        info.rank = int(env["OMPI_COMM_WORLD_RANK"])
        info.local_rank = int(env.get("OMPI_COMM_WORLD_LOCAL_RANK", "0"))
        info.master_addr = env.get("MASTER_ADDR", "127.0.0.1")
        info.master_port = int(env.get("MASTER_PORT", "29500"))
    elif "PMI_SIZE" in env and "PMI_RANK" in env:
        info.world = int(env["PMI_SIZE"])
        info.rank = int(env["PMI_RANK"])
        info.local_rank = int(env.get("MPI_LOCALRANKID", env.get("PMI_LOCAL_RANK", "0")))
        info.master_addr = env.get("MASTER_ADDR", "127.0.0.1")
        info.master_port = int(env.get("MASTER_PORT", "29500"))
    elif "SLURM_NTASKS" in env and "SLURM_PROCID" in env and int(env["SLURM_NTASKS"]) > 1:
        info.world = int(env["SLURM_NTASKS"])
        info.rank = int(env["SLURM_PROCID"])
        info.local_rank = int(env.get("SLURM_LOCALID", "0"))
        info.master_addr = env.get("MASTER_ADDR", env.get("SLURM_LAUNCH_NODE_IPADDR", "127.0.0.1"))
        info.master_port = int(env.get("MASTER_PORT", "29500"))
    else:
        info.role = "serial"
    if getattr(flags, "master_addr", ""):
        info.master_addr = flags.master_addr
    if gpu:
        import torch
        ndev = torch.cuda.device_count()
        info.device = f"cuda:{info.local_rank % ndev}"
        info.backend = "nccl"
    else:
        info.device = "cpu"
        info.backend = "gloo"
    return info


def init_process_group(info: ClusterInfo, timeout_s: int = 1800):
    """torch.distributed bootstrap (TCPStore rendezvous at master_addr:master_port)."""
    if not info.distributed:
        return None
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        return dist.group.WORLD
    kw = {}
    if info.backend == "nccl":
        torch.cuda.set_device(torch.device(info.device))
        kw["device_id"] = torch.device(info.device)
    dist.init_process_group(info.backend, init_method=f"tcp://{info.master_addr}:{info.master_port}",
                            rank=info.rank, world_size=info.world, timeout=timedelta(seconds=timeout_s), **kw)
    log.info("rank %d/%d up (backend %s, device %s)", info.rank, info.world, info.backend, info.device)
    return dist.group.WORLD
