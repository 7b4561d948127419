"""Collective watchdog: a host thread that aborts a rank whose gradient exchange stalls.

The reference has no failure detection: SyncReplicasOptimizer needs every replica each step, so
one dead worker stalls the whole job until someone runs kill.sh. Here each step's
exchange is bracketed by the data-parallel engine: `arm(step)` when the backward pass starts
issuing collectives, `done(event)` once the host has queued the final waits (with a device event
that completes when the last bucket has been reduced). The thread aborts the process when either

  * the host is still inside the exchange `timeout_s` after arming (a blocking gloo collective,
    or a P2P wait whose peer never arrived), or
  * the device event has not completed `timeout_s` after `done` (an RCCL kernel stuck on a dead
    peer),

so the launcher (`parallel/launch.py --max_restarts`) sees a non-zero exit, tears the group
down and restarts every rank from the latest checkpoint. The process-group timeout
(`--collective_timeout_secs`, passed to init_process_group) backs this up inside RCCL itself.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Optional

log = logging.getLogger("drn")

EXIT_CODE = 3


def _abort(msg: str):
    log.error(msg)
    logging.shutdown()
    os._exit(EXIT_CODE)


class CollectiveWatchdog:
    def __init__(self, timeout_s: float, on_timeout: Optional[Callable[[str], None]] = None, poll_s: float = 0.5,
                 rank: int = 0):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout or _abort
        self.poll_s = poll_s
        self.rank = rank
        self._lock = threading.Lock()
        self._step = None
        self._t_arm = 0.0
        self._t_done = None
        self._event = None
        self._fired = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="drn-collective-watchdog", daemon=True)
        self._thread.start()

    def arm(self, step: int):
        with self._lock:
            self._step, self._t_arm, self._t_done, self._event = step, time.monotonic(), None, None

    def done(self, event=None):
        with self._lock:
            self._t_done, self._event = time.monotonic(), event

    def disarm(self):
        with self._lock:
            self._step = None

    def close(self):
        self._stop.set()
        self._thread.join(timeout=5)

    @property
    def fired(self) -> bool:
        return self._fired

    def _check(self) -> Optional[str]:
        with self._lock:
            if self._step is None or self._fired:
                return None
            now = time.monotonic()
            if self._t_done is None:
                if now - self._t_arm > self.timeout_s:
                    return (f"rank {self.rank}: gradient exchange of step {self._step} still blocked on the host "
                            f"after {now - self._t_arm:.1f} s (a peer rank is gone or stuck)")
                return None
            ev = self._event
            if ev is not None and now - self._t_done > self.timeout_s and not ev.query():
                return (f"rank {self.rank}: all-reduce of step {self._step} has not completed on the device "
                        f"{now - self._t_done:.1f} s after it was queued (RCCL/P2P collective stalled)")
            if ev is None or ev.query():
                self._step = None
            return None

    def _run(self):
        while not self._stop.wait(self.poll_s):
            msg = self._check()
            if msg:
                self._fired = True
                self.on_timeout(msg)
