"""Entry-point dispatch shared by the top-level scripts (resnet_cifar_main.py & co.).

Each reference script keeps its name, flag defaults and behaviour:
  resnet_cifar_main.py          CIFAR train; serial / --job_name worker (PS-mode flags) / torchrun
  resnet_cifar_main_horovod.py  CIFAR train with the all-reduce engine forced on (Horovod analog;
                                SURVEY Q15: the reference trained independent replicas without
                                --use_horovod=True)
  resnet_imagenet_main.py       ImageNet train (default --dataset=imagenet)
  resnet_cifar_eval.py          CIFAR eval poller (batch 100, --mode=eval)
  resnet_imagenet_eval.py       ImageNet eval poller
  resnet_single.py              single-process train (+ --mode=eval) — the reference version is
                                stale and crashes; this one works (BASELINE config 1)
"""
from __future__ import annotations

import sys

from . import flags as flags_mod


def _flags(**defaults):
    fv = flags_mod.FlagValues()
    flags_mod.define_reference_flags(fv, **defaults)
    return fv


# per-entry-point flag defaults (the reference scripts' own DEFINE_* defaults)
ENTRY_DEFAULTS = {
    "cifar_main": dict(dataset="cifar10", batch_size=32, train_steps=2000, log_every_n_steps=20),
    "cifar_horovod_main": dict(dataset="cifar10", batch_size=32, train_steps=2000, log_every_n_steps=20,
                               use_horovod=True),
    "imagenet_main": dict(dataset="imagenet", batch_size=128, train_steps=200, log_every_n_steps=40,
                          image_size=224, num_epochs=90),
    "cifar_eval_main": dict(dataset="cifar10", mode="eval"),
    "imagenet_eval_main": dict(dataset="imagenet", mode="eval", batch_size=128, num_epochs=3000, image_size=224),
    "single_main": dict(dataset="cifar10", batch_size=128, train_steps=2000, log_every_n_steps=100,
                        resnet_size=20),
}


def entry_flags(entry: str, argv=None):
    """Parsed flags of an entry point (`argv` without the program name)."""
    FLAGS = _flags(**ENTRY_DEFAULTS[entry])
    FLAGS([entry] + list(sys.argv[1:] if argv is None else argv))
    return FLAGS


def cifar_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["cifar_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    from .train.trainer import train
    if FLAGS.mode != "train":
        raise SystemExit("resnet_cifar_main.py trains; use resnet_cifar_eval.py --mode=eval to evaluate")
    return train(FLAGS)


def cifar_horovod_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["cifar_horovod_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    FLAGS.use_horovod = True
    from .train.trainer import train
    return train(FLAGS)


def imagenet_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["imagenet_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    from .train.trainer import train
    return train(FLAGS)


def cifar_eval_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["cifar_eval_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    from .train.evaluator import evaluate
    evaluate(FLAGS, eval_batch_size=100)
    return 0


def imagenet_eval_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["imagenet_eval_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    from .train.evaluator import evaluate
    evaluate(FLAGS, eval_batch_size=FLAGS.batch_size)
    return 0


def single_main(argv=None):
    FLAGS = _flags(**ENTRY_DEFAULTS["single_main"])
    FLAGS(list(sys.argv if argv is None else argv))
    if FLAGS.mode == "eval":
        from .train.evaluator import evaluate
        evaluate(FLAGS, eval_batch_size=100)
        return 0
    FLAGS.job_name = None
    from .train.trainer import train
    return train(FLAGS)
