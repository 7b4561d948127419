"""Persistent kernel-selection database: the analog of MIOpen's find-db / perf-db.

The HIP backend picks a kernel configuration per convolution geometry by timing candidates
(ops/backend.py `_tune_conv`, `_tune_wgrad`). Timing is noisy (clock ramps, neighbours' cache
state), so two runs of the same library could pick different tiles and differ by several percent
(CIFAR bs32: 1.77-1.95 ms across runs). The choices are therefore persisted and reused: a
geometry found in the database is never re-timed, so runs of one library are deterministic and
start without the tuning pass.

Entries are keyed by
  * the device architecture (gcnArchName, e.g. ``gfx950:sramecc+:xnack-``) and CU count,
  * the hash of the sources the choices depend on (``drn_tune_hash``, ops/build.py: the conv,
    weight-gradient and stem kernels + shared headers): a library with other conv kernels never
    reuses stale choices, while edits of unrelated kernels (pooling, SGD, BN applies) keep them,
  * the geometry key the backend already uses (conv_key / wgrad_key).

Two files, as MIOpen keeps a system and a user database:
  * the SYSTEM database ``ops/tune_db.json`` ships with the tree (built on an MI355X by
    scripts/make_tune_db.py) and is only ever READ: no run, test or bench rewrites it;
  * the USER database ``DRN_TUNE_DB`` (default ``~/.cache/drn/tune_db.json``) receives every
    choice this process timed itself; it is consulted for geometries the system database lacks.
``DRN_TUNE_DB=off`` disables both; ``DRN_TUNE_DB_SYSTEM=off`` disables only the system database
(scripts/make_tune_db.py rebuilds the shipped file that way, so every geometry is re-timed and
the output holds the complete section, not just what the shipped file lacked). Writes are read-merge-write through a temporary file and
``os.replace`` (several ranks of one node may write concurrently; the last rename wins, every
version is a complete file). Sections of other library hashes are dropped when a section is
written (they can never match again).
"""
from __future__ import annotations

import json
import os
import threading
from pathlib import Path
from typing import Optional

VERSION = 1
SYSTEM_PATH = Path(__file__).resolve().parent / "tune_db.json"
_LOCK = threading.Lock()


def enabled() -> bool:
    return os.environ.get("DRN_TUNE_DB", "").lower() not in ("off", "0", "none")


def system_enabled() -> bool:
    return enabled() and os.environ.get("DRN_TUNE_DB_SYSTEM", "").lower() not in ("off", "0", "none")


def db_path() -> Optional[Path]:
    """The writable user database (None when disabled)."""
    if not enabled():
        return None
    p = os.environ.get("DRN_TUNE_DB", "")
    return Path(p) if p else Path(os.path.expanduser("~")) / ".cache" / "drn" / "tune_db.json"


def _load_section(path: Optional[Path], section: str) -> tuple:
    if path is None or not path.exists():
        return {}, {}
    try:
        data = json.loads(path.read_text())
        sec = data.get("sections", {}).get(section, {}) if data.get("version") == VERSION else {}
        return dict(sec.get("conv", {})), dict(sec.get("wgrad", {}))
    except (OSError, ValueError):
        return {}, {}


def _key(t) -> str:
    return ",".join(str(int(v)) if isinstance(v, (bool, int)) else str(v) for v in t)


class TuneDB:
    """One section (device + library) of the databases: lookups read the system database first,
    then the user database; new choices go to the user database only."""

    def __init__(self, section: str, path: Optional[Path] = None, system: Optional[Path] = None):
        self.section = section
        self.path = db_path() if path is None else path
        on = system_enabled() or (path is not None and system is not None)
        self.sys_conv, self.sys_wgrad = _load_section(SYSTEM_PATH if system is None else system, section) if on \
            else ({}, {})
        self.conv, self.wgrad = _load_section(self.path, section)  # this process's / the user's choices
        self.dirty = False

    # conv: (config id, split-K factor / -stream-K grid)
    def get_conv(self, key) -> Optional[tuple]:
        k = _key(key)
        v = self.sys_conv.get(k, self.conv.get(k))
        return (int(v[0]), int(v[1])) if v is not None else None

    def put_conv(self, key, val) -> None:
        self.conv[_key(key)] = [int(val[0]), int(val[1])]
        self.dirty = True

    # wgrad: (split target, pipeline, atomic, min steps)
    def get_wgrad(self, key) -> Optional[tuple]:
        k = _key(key)
        v = self.sys_wgrad.get(k, self.wgrad.get(k))
        return (int(v[0]), int(v[1]), bool(v[2]), int(v[3])) if v is not None else None

    def put_wgrad(self, key, val) -> None:
        self.wgrad[_key(key)] = [int(val[0]), int(val[1]), bool(val[2]), int(val[3])]
        self.dirty = True

    def save(self) -> bool:
        """Merge this section into the user database (entries already on disk for this section
        are kept unless this process has its own choice for the same key). The system database
        is never written. Returns True if written."""
        if self.path is None or not self.dirty or self.path.resolve() == SYSTEM_PATH.resolve():
            return False
        with _LOCK:
            self.path.parent.mkdir(parents=True, exist_ok=True)
            data = {"version": VERSION, "sections": {}}
            if self.path.exists():
                try:
                    old = json.loads(self.path.read_text())
                    if old.get("version") == VERSION:
                        data = old
                except (OSError, ValueError):
                    pass
            arch = self.section.split("|", 1)[0]
            # drop sections of other library builds on this device (never valid again)
            secs = {k: v for k, v in data.get("sections", {}).items()
                    if k == self.section or k.split("|", 1)[0] != arch}
            sec = secs.get(self.section, {"conv": {}, "wgrad": {}})
            sec["conv"] = {**sec.get("conv", {}), **self.conv}
            sec["wgrad"] = {**sec.get("wgrad", {}), **self.wgrad}
            secs[self.section] = sec
            data["sections"] = secs
            tmp = self.path.with_name(f".{self.path.name}.{os.getpid()}.tmp")
            try:
                tmp.write_text(json.dumps(data, indent=0, sort_keys=True))
                os.replace(tmp, self.path)
            except OSError:
                try:
                    tmp.unlink()
                except OSError:
                    pass
                return False
            self.dirty = False
            return True


def section_for(device, lib_handle) -> str:
    """Section name: device architecture + CU count + library source hash."""
    import ctypes

    import torch
    props = torch.cuda.get_device_properties(device)
    arch = getattr(props, "gcnArchName", props.name)
    h = "nohash"
    for sym in ("drn_tune_hash", "drn_src_hash"):  # tuning-relevant sources; older libraries: all
        if hasattr(lib_handle, sym):
            f = getattr(lib_handle, sym)
            f.restype, f.argtypes = ctypes.c_char_p, []
            h = f().decode()[:16]
            break
    return f"{arch}/{props.multi_processor_count}cu|{h}"
