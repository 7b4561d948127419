"""`evaluate()` checkpoint poller (reference resnet_cifar_eval.py:85-141,
resnet_imagenet_eval.py:154-210): restore the latest checkpoint in --log_root, run
--eval_batch_count batches in inference mode (BN moving statistics), log
`loss, precision, best precision`, write `Precision` / `Best Precision` summaries at the
checkpoint's global step, sleep and repeat unless --eval_once.

Fixes of reference quirks: no busy-spin when there is no checkpoint (Q8), best precision
persisted in eval_dir/best_precision.json across restarts (Q11), the eval set is read in order
(a --eval_batch_count covering the set is a full deterministic pass, Q10).
"""
from __future__ import annotations

import json
import logging
import os
import time

import torch

from ..ckpt.saver import Saver, latest_checkpoint, step_of
from ..parallel import cluster as cl
from ..runtime.executor import Executor
from ..runtime.state import import_state
from ..utils.events import EventFileWriter
from .session import make_backend
from .trainer import WEIGHT_DECAY, apply_thread_flags, make_feeder, model_spec_from_flags, setup_logging

log = logging.getLogger("drn")


def _load_best(path):
    try:
        return float(json.load(open(path))["best_precision"])
    except Exception:
        return 0.0


def evaluate(FLAGS, eval_batch_size: int = 100, max_evals: int = -1):
    setup_logging(0)
    apply_thread_flags(FLAGS)
    if FLAGS.mode != "eval":
        raise ValueError("this entry point only evaluates: pass --mode=eval (the reference called an "
                         "undefined train() here, SURVEY Q1)")
    FLAGS.job_name = None
    cluster = cl.resolve(FLAGS, env={})
    spec = model_spec_from_flags(FLAGS)
    be = make_backend(cluster.device, getattr(FLAGS, "precision", "bf16"))
    ex = Executor(spec, eval_batch_size, be, cluster.device, weight_decay=WEIGHT_DECAY.get(FLAGS.dataset, 1e-4))
    writer = EventFileWriter(FLAGS.eval_dir) if FLAGS.eval_dir else None
    best_path = os.path.join(FLAGS.eval_dir, "best_precision.json") if FLAGS.eval_dir else None
    best = _load_best(best_path) if best_path else 0.0
    last = None
    n_eval = 0
    results = []
    while True:
        prefix = latest_checkpoint(FLAGS.log_root)
        if prefix is None:
            log.info("No model to eval yet at %s", FLAGS.log_root)
        elif prefix == last and not FLAGS.eval_once:
            pass
        else:
            try:
                import_state(ex, Saver.restore(prefix))
            except (OSError, ValueError, KeyError) as e:  # half-written / rotated away: retry later
                log.warning("Cannot restore checkpoint %s: %s", prefix, e)
                prefix = None
            if prefix is not None:
                last = prefix
                step = ex.P.global_step or step_of(prefix)
                feeder = make_feeder(FLAGS, ex, cluster, False, batch=eval_batch_size)
                total_loss, correct, total = 0.0, 0, 0
                try:
                    for _ in range(FLAGS.eval_batch_count):
                        if not feeder.next():
                            break
                        ex.forward(train=False)
                        v = int(getattr(feeder, "valid", ex.N))  # wrapped padding of a final partial batch
                        feeder.prefetch()   # host load of the next batch while this one runs
                        total_loss += float(ex.loss_vec[:v].double().sum())
                        correct += int(ex.correct[:v].sum())
                        total += v
                finally:
                    feeder.close()
                precision = correct / max(total, 1)
                loss = total_loss / max(total, 1) + ex.wd * float(ex.P.trainable_l2())
                best = max(best, precision)
                if writer is not None:
                    writer.add_scalars(step, {"Precision": precision, "Best Precision": best})
                    writer.flush()
                if best_path:
                    tmp = best_path + ".tmp"
                    with open(tmp, "w") as f:
                        json.dump({"best_precision": best, "step": step}, f)
                    os.replace(tmp, best_path)
                log.info("loss: %.3f, precision: %.3f, best precision: %.3f", loss, precision, best)
                results.append({"step": step, "loss": loss, "precision": precision, "best_precision": best})
                n_eval += 1
        if FLAGS.eval_once and last is not None:
            break
        if 0 <= max_evals <= n_eval:
            break
        time.sleep(max(1, FLAGS.eval_interval_secs))
    if writer is not None:
        writer.close()
    return results
