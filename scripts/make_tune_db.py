#!/usr/bin/env python3
"""Build the kernel-selection database (ops/tunedb.py) for the benchmark configurations with a
more thorough tuner (more launches per candidate, more finalists, more re-timing rounds) than
the per-run autotuner, so every run of this library picks the same, carefully timed kernels.

usage (on the GPU box): DRN_TUNE_DB=<out.json> python scripts/make_tune_db.py
The resulting file is copied to distributed_resnet_tensorflow_amd/ops/tune_db.json (it is keyed
by the library's source hash: rebuild it whenever a kernel source changes).
"""
import os
import sys

# every geometry re-timed: the shipped (system) database is not consulted while rebuilding it
os.environ["DRN_TUNE_DB_SYSTEM"] = "off"
os.environ.setdefault("DRN_TUNE_ITERS", "20")
os.environ.setdefault("DRN_TUNE_TOP", "4")        # (more finalists made the in-situ pick noisier)
os.environ.setdefault("DRN_INSITU_ROUNDS", "3")
os.environ.setdefault("DRN_TUNE_ROUNDS", "4")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.models.spec import build_spec  # noqa: E402
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend  # noqa: E402
from distributed_resnet_tensorflow_amd.runtime.executor import Executor  # noqa: E402

CONFIGS = [("imagenet", 50, 128, 1), ("cifar10", 50, 128, 1), ("cifar10", 50, 32, 1), ("imagenet", 50, 256, 2)]
for ds, depth, bs, width in CONFIGS:
    be = HipBackend("cuda")
    ex = Executor(build_spec(ds, depth, width=width), bs, be, "cuda", seed=1234,
                  weight_decay=1e-4 if ds == "imagenet" else 2e-4)
    be.synthetic_images(ex.images, seed=17)
    ex.autotune()  # tunes every launch of the step and saves the new entries
    print(f"{ds} resnet{depth} x{width} bs{bs}: {len(be.conv_cfg)} conv + {len(be.wgrad_ns)} wgrad choices, "
          f"{be.db_hits} database hits", flush=True)
    del ex, be
    torch.cuda.empty_cache()
