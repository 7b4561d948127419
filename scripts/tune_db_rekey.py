#!/usr/bin/env python3
"""Carry the shipped kernel-selection database over a kernel-source edit that leaves the tuned
kernels untouched.

The database section is keyed by the hash of the tuning sources (ops/build.py tune_hash): any edit
of conv_fwd.hip / conv_wgrad.hip / stem.hip or a shared header retires every shipped choice, and a
fresh rebuild re-times all of them (with its own run-to-run noise). When an edit only ADDS a kernel
(e.g. a new weight-gradient pipeline) the existing choices stay valid: this script re-keys the
newest section to the current hash and drops the entries the new code can improve, so those -- and
only those -- are tuned again (by the next run, or thoroughly by scripts/make_tune_db.py pointed at
the result with DRN_TUNE_DB_SYSTEM=off).

    python scripts/tune_db_rekey.py [--drop-wgrad KEYPREFIX ...] [--drop-conv KEYPREFIX ...] [--out PATH]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_resnet_tensorflow_amd.ops import build  # noqa: E402
from distributed_resnet_tensorflow_amd.ops.tunedb import SYSTEM_PATH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--db", default=str(SYSTEM_PATH))
    ap.add_argument("--out", default="")
    ap.add_argument("--drop-wgrad", nargs="*", default=[])
    ap.add_argument("--drop-conv", nargs="*", default=[])
    a = ap.parse_args()
    data = json.load(open(a.db))
    new_hash = build.tune_hash()[:16]
    (old_key, sec), = list(data["sections"].items())[-1:]
    dev = old_key.split("|")[0]
    conv = {k: v for k, v in sec["conv"].items() if not any(k.startswith(p) for p in a.drop_conv)}
    wgrad = {k: v for k, v in sec["wgrad"].items() if not any(k.startswith(p) for p in a.drop_wgrad)}
    data["sections"] = {f"{dev}|{new_hash}": {"conv": conv, "wgrad": wgrad}}
    out = a.out or a.db
    open(out, "w").write(json.dumps(data, indent=0, sort_keys=True))  # (tunedb.py's format)
    print(f"{old_key} -> {dev}|{new_hash}: {len(conv)} conv ({len(sec['conv']) - len(conv)} dropped), "
          f"{len(wgrad)} wgrad ({len(sec['wgrad']) - len(wgrad)} dropped) -> {out}")


if __name__ == "__main__":
    main()
