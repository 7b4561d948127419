"""Local multi-process launcher with failure detection and restart-from-checkpoint.

    python -m distributed_resnet_tensorflow_amd.parallel.launch --nproc 8 [--max_restarts 3] \
        resnet_imagenet_main.py --num_gpus=8 --log_root=/ckpt ...

One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in
the environment; the entry point pins GPU LOCAL_RANK). The reference relied on Slurm `srun
--no-kill` and manual restarts (scripts/run_dist_tf_daint.sh:200-204) and its
SyncReplicas job stalled forever when a worker died; here a dead rank tears the whole group
down (no rank is left blocked in a collective) and the job is relaunched up to --max_restarts
times; every rank resumes from the latest complete checkpoint in --log_root (atomic writes,
state file written last). Processes are managed by exact PID / process group, never by name.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(nproc: int, cmd: List[str], port: int, base_env: dict, nnodes: int = 1, node_rank: int = 0,
           log_dir: str = "", tag: str = "", pid_file: str = "") -> List[subprocess.Popen]:
    procs = []
    world = nproc * nnodes
    host = socket.gethostname()
    for lr in range(nproc):
        r = node_rank * nproc + lr
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(lr), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(nproc),
                   NODE_RANK=str(node_rank), MASTER_ADDR=env.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=str(port))
        out = None
        if log_dir:
            # per-process log, named like the reference launcher's worker.$JOB.$host-port.log
            os.makedirs(log_dir, exist_ok=True)
            out = open(os.path.join(log_dir, f"worker.{tag or 'job'}.{host}-{r}.log"), "ab")
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True, stdout=out,
                                      stderr=subprocess.STDOUT if out else None))
        if out:
            out.close()
    if pid_file:
        with open(pid_file, "a") as f:
            for p in procs:
                f.write(f"{p.pid}\n")
    return procs


def _kill_all(procs, grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t0 = time.time()
    for p in procs:
        try:
            p.wait(timeout=max(0.1, grace - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run(nproc: int, cmd: List[str], max_restarts: int = 0, poll: float = 0.5, nnodes: int = 1, node_rank: int = 0,
        log_dir: str = "", tag: str = "", pid_file: str = "") -> int:
    """Run nproc ranks of `cmd` on this node (ranks node_rank*nproc ... of nnodes*nproc).
    Multi-node jobs need a fixed MASTER_ADDR/MASTER_PORT (the first node); a failed rank ends
    this node's ranks and the launcher exits non-zero (resubmission resumes from the
    checkpoint); single-node jobs restart in place up to max_restarts times."""
    base_env = dict(os.environ)
    attempt = 0
    if nnodes > 1 and not base_env.get("MASTER_PORT"):
        raise SystemExit("multi-node launch needs MASTER_ADDR and MASTER_PORT")
    while True:
        port = int(base_env.get("MASTER_PORT", "0")) or _free_port()
        procs = _spawn(nproc, cmd, port, base_env, nnodes, node_rank, log_dir, tag, pid_file)
        failed = None
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    failed = bad[0]
                    break
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(poll)
        except KeyboardInterrupt:
            _kill_all(procs)
            return 130
        rank, code = failed
        print(f"[drn.launch] rank {rank} exited with code {code}; tearing down the job", file=sys.stderr, flush=True)
        _kill_all(procs)
        if attempt >= max_restarts or nnodes > 1:
            return code if code > 0 else 1
        attempt += 1
        print(f"[drn.launch] restart {attempt}/{max_restarts} (resuming from the latest checkpoint)",
              file=sys.stderr, flush=True)
        base_env.pop("MASTER_PORT", None)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node_rank", type=int, default=0)
    ap.add_argument("--master_addr", default=None)
    ap.add_argument("--master_port", type=int, default=0)
    ap.add_argument("--log_dir", default="", help="write worker.<tag>.<host>-<rank>.log files here")
    ap.add_argument("--tag", default="", help="job tag used in log file names (e.g. $SLURM_JOB_ID)")
    ap.add_argument("--pid_file", default="", help="append child PIDs here (scripts/kill.sh reads it)")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.master_addr:
        os.environ["MASTER_ADDR"] = a.master_addr
    if a.master_port:
        os.environ["MASTER_PORT"] = str(a.master_port)
    cmd = [sys.executable, a.script] + a.args
    return run(a.nproc, cmd, a.max_restarts, nnodes=a.nnodes, node_rank=a.node_rank, log_dir=a.log_dir,
               tag=a.tag, pid_file=a.pid_file)


if __name__ == "__main__":
    sys.exit(main())
