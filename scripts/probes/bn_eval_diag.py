#!/usr/bin/env python3
"""Why does a checkpoint with training precision 1.0 evaluate lower? Evaluates one CIFAR
checkpoint on a record set three ways, all on the same eval-preprocessed batches:
  moving  -- inference mode, BN moving statistics (what resnet_cifar_eval.py reports);
  batch   -- BN with the batch's own statistics (training-mode normalisation, no update);
  recal   -- moving statistics re-estimated for the CURRENT weights (mean of per-batch
             statistics over the set), then inference mode.
moving << batch ~ recal means the moving averages lag the weights (training-schedule effect),
not a wrong eval path.
    python scripts/probes/bn_eval_diag.py <log_root> '<records glob>' [resnet_size]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_resnet_tensorflow_amd.ckpt.saver import Saver, latest_checkpoint  # noqa: E402
from distributed_resnet_tensorflow_amd.data import cifar as cifar_data  # noqa: E402
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2  # noqa: E402
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend  # noqa: E402
from distributed_resnet_tensorflow_amd.runtime.executor import Executor  # noqa: E402
from distributed_resnet_tensorflow_amd.runtime.state import import_state  # noqa: E402
from distributed_resnet_tensorflow_amd.train.feeder import CifarFeeder  # noqa: E402


def main():
    log_root, pattern = sys.argv[1], sys.argv[2]
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    ex = Executor(cifar_resnet_v2(size), 100, HipBackend(), "cuda")
    import_state(ex, Saver.restore(latest_checkpoint(log_root)))
    import glob
    recs = cifar_data.CifarRecords(sorted(glob.glob(pattern)))
    nb = max(1, recs.n // 100)

    def batches():
        ld = cifar_data.CifarLoader(recs, 100, False, pin=True, pin_device=torch.device("cuda"))
        fd = CifarFeeder(ex, ld, False)
        for _ in range(nb):
            fd.next()
            yield
        fd.close()

    saved = ex.P.bn_state.clone()

    def run(train: bool):
        c = t = 0
        for _ in batches():
            ex.forward(train=train)
            c += int(ex.correct.sum())
            t += ex.N
            if train:
                ex.P.bn_state.copy_(saved)  # batch statistics, no moving-average side effect
        return c / t

    moving = run(False)
    batch = run(True)
    # re-estimate: average of per-batch mean / variance for the current weights
    acc = torch.zeros_like(saved)
    k = 0
    for _ in batches():
        ex.P.bn_state.copy_(saved)
        before = ex.P.bn_state.clone()
        ex.forward(train=True)
        # one update: new = d*old + (1-d)*batch  ->  batch = (new - d*old) / (1-d)
        acc += (ex.P.bn_state - 0.997 * before) / 0.003
        k += 1
    ex.P.bn_state.copy_(acc / k)
    recal = run(False)
    ex.P.bn_state.copy_(saved)
    print(f"{log_root}: moving {moving:.3f}  batch {batch:.3f}  recalibrated {recal:.3f}", flush=True)


if __name__ == "__main__":
    main()
