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


def _spawn(nproc: int, cmd: List[str], port: int, base_env: dict) -> List[subprocess.Popen]:
    procs = []
    for r in range(nproc):
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR=env.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
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


def run(nproc: int, cmd: List[str], max_restarts: int = 0, poll: float = 0.5) -> int:
    base_env = dict(os.environ)
    attempt = 0
    while True:
        port = int(base_env.get("MASTER_PORT", "0")) or _free_port()
        procs = _spawn(nproc, cmd, port, base_env)
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
        if attempt >= max_restarts:
            return code if code > 0 else 1
        attempt += 1
        print(f"[drn.launch] restart {attempt}/{max_restarts} (resuming from the latest checkpoint)",
              file=sys.stderr, flush=True)
        base_env.pop("MASTER_PORT", None)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, a.script] + a.args
    return run(a.nproc, cmd, a.max_restarts)


if __name__ == "__main__":
    sys.exit(main())
