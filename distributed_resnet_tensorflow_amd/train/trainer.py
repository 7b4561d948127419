"""`train()` of the reference entry points (resnet_cifar_main.py:250-337,
resnet_imagenet_main.py:185-263, resnet_cifar_main_horovod.py:249-339), on the MI355X engine."""
from __future__ import annotations

import json
import logging
import os
import sys

import torch

from ..data import cifar as cifar_data
from ..models.spec import build_spec
from ..parallel import cluster as cl
from ..utils.events import EventFileWriter
from ..utils.profiler import model_report
from . import lr as lr_mod
from .feeder import CifarFeeder, ImagenetFeeder, SyntheticFeeder
from .hooks import (CheckpointHook, FaultInjectHook, LoggingHook, ProfileHook, StopAtStepHook, SummaryHook)
from .session import TrainingSession

log = logging.getLogger("drn")

WEIGHT_DECAY = {"cifar10": 2e-4, "cifar100": 2e-4, "imagenet": 1e-4}


def setup_logging(rank: int = 0):
    fmt = f"%(asctime)s [rank {rank}] %(levelname)s %(message)s" if rank else "%(asctime)s %(levelname)s %(message)s"
    logging.basicConfig(level=logging.INFO, format=fmt, stream=sys.stdout, force=True)


def apply_thread_flags(FLAGS):
    if FLAGS.num_intra_threads > 0:
        torch.set_num_threads(FLAGS.num_intra_threads)
    if FLAGS.num_inter_threads > 0:
        try:
            torch.set_num_interop_threads(FLAGS.num_inter_threads)
        except RuntimeError:
            pass


def model_spec_from_flags(FLAGS):
    ds = FLAGS.dataset
    model = FLAGS.model if FLAGS.model != "lrnet" else "resnet"
    # --width_multiplier only shapes --model=wide_resnet; --model=resnet is always the reference's
    # ResNet-v2 (resnet_model.py:74, resnet_imagenet_main.py:266-272: 25,551,401 params at size 50)
    width = FLAGS.width_multiplier if model == "wide_resnet" else 1
    return build_spec(ds, FLAGS.resnet_size, model=model, width=width)


def _meta(FLAGS, spec):
    return {"dataset": FLAGS.dataset, "resnet_size": FLAGS.resnet_size, "model": FLAGS.model,
            "width_multiplier": FLAGS.width_multiplier if FLAGS.model == "wide_resnet" else 1,
            "num_classes": spec.num_classes,
            "spec_name": spec.name}


def make_feeder(FLAGS, ex, cluster, is_training: bool, data_state=None, batch=None):
    bs = batch or ex.N
    if FLAGS.synthetic_data:
        return SyntheticFeeder(ex, seed=FLAGS.seed + 101 * cluster.rank)
    ds = data_state or {}
    gpu = ex.device.type == "cuda"
    pin = dict(pin=gpu, pin_device=ex.device if gpu else None)
    if FLAGS.dataset in ("cifar10", "cifar100"):
        path = FLAGS.train_data_path if is_training else FLAGS.eval_data_path
        recs = cifar_data.CifarRecords(cifar_data.get_filenames(is_training, path, FLAGS.dataset), FLAGS.dataset)
        loader = cifar_data.CifarLoader(recs, bs, is_training, seed=FLAGS.seed, rank=cluster.rank,
                                        world=cluster.world, epoch=int(ds.get("data_epoch", 0)),
                                        cursor=int(ds.get("data_cursor", 0)), **pin)
        return CifarFeeder(ex, loader, is_training)
    from ..data import imagenet
    path = FLAGS.train_data_path if is_training else FLAGS.eval_data_path
    loader = imagenet.ImagenetLoader(path, bs, is_training, seed=FLAGS.seed, rank=cluster.rank, world=cluster.world,
                                     num_threads=max(2, FLAGS.num_workers * 4),
                                     num_epochs=FLAGS.num_epochs if is_training else 1,
                                     epoch=int(ds.get("data_epoch", 0)), cursor=int(ds.get("data_cursor", 0)),
                                     batch_index=int(ds.get("data_batch", 0)), workers=FLAGS.input_workers, **pin)
    return ImagenetFeeder(ex, loader, is_training)


def train(FLAGS, cluster=None):
    cluster = cluster or cl.resolve(FLAGS)
    setup_logging(cluster.rank)
    apply_thread_flags(FLAGS)
    if cluster.role == "ps":
        log.info("job_name=ps: parameter servers are not used by the all-reduce engine; exiting")
        return 0
    if FLAGS.model == "lrnet":
        from ..models.lrnet import train_lrnet
        return train_lrnet(FLAGS, cluster)
    cl.init_process_group(cluster, timeout_s=FLAGS.collective_timeout_secs)
    torch.manual_seed(FLAGS.seed)
    spec = model_spec_from_flags(FLAGS)
    if cluster.is_chief:
        log.info(model_report(spec))
    wd = FLAGS.weight_decay if FLAGS.weight_decay is not None else WEIGHT_DECAY.get(FLAGS.dataset, 1e-4)
    # reference: SyncReplicas iff --job_name given and --sync_replicas; Horovod always averages
    sync_mode = "sync"
    if FLAGS.job_name == "worker" and not FLAGS.sync_replicas and not FLAGS.use_horovod:
        sync_mode = "delayed"
        if cluster.is_chief:
            log.info("--sync_replicas=False: 1-step-delayed all-reduce (async-PS analog, staleness 1; not "
                     "bit-equivalent to TF asynchronous parameter servers)")
    sess = TrainingSession(spec, FLAGS.batch_size, cluster, weight_decay=wd, lr_schedule=lr_mod.for_dataset(FLAGS.dataset, FLAGS.lr_schedule_scale),
                           checkpoint_dir=FLAGS.log_root, max_to_keep=FLAGS.max_to_keep, seed=FLAGS.seed,
                           use_graph=FLAGS.hip_graph, sync_mode=sync_mode, bucket_mb=FLAGS.bucket_mb,
                           meta=_meta(FLAGS, spec), allreduce=FLAGS.allreduce, wire=FLAGS.allreduce_wire,
                           collective_timeout_s=FLAGS.collective_timeout_secs, precision=FLAGS.precision,
                           shard_optimizer=FLAGS.optimizer_sharding)
    feeder = make_feeder(FLAGS, sess.ex, cluster, True, sess.data_state)
    is_imagenet = FLAGS.dataset == "imagenet"
    hooks = [LoggingHook(FLAGS.log_every_n_steps, FLAGS.batch_size * cluster.world,
                         metrics_path=os.path.join(FLAGS.log_root, "metrics.jsonl") if (FLAGS.log_root and cluster.is_chief) else None,
                         with_lr=not is_imagenet, world=cluster.world),
             StopAtStepHook(FLAGS.train_steps)]
    if FLAGS.fault_inject_step >= 0:
        hooks.append(FaultInjectHook(FLAGS.fault_inject_step, FLAGS.fault_inject_rank, cluster.rank))
    chief_hooks = []
    summary_dir = FLAGS.train_dir if is_imagenet else FLAGS.eval_dir  # reference quirk, :276 / :213
    if summary_dir and FLAGS.save_summaries_steps > 0:
        chief_hooks.append(SummaryHook(EventFileWriter(summary_dir), FLAGS.save_summaries_steps))
    if FLAGS.log_root:
        save_fn = lambda step, blocking: sess.save(step, blocking)  # noqa: E731
        if sess.sharded:  # collective save: every rank gathers its optimizer shards
            hooks.append(CheckpointHook(FLAGS.save_checkpoint_secs, save_fn, agree=sess.engine.agree))
        else:
            chief_hooks.append(CheckpointHook(FLAGS.save_checkpoint_secs, save_fn))
    if FLAGS.profile_steps:
        chief_hooks.append(ProfileHook(FLAGS.profile_steps, FLAGS.log_root or "."))
    try:
        sess.run(feeder, hooks, chief_hooks)
    finally:
        feeder.close()
    if cluster.distributed:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    log.info("training finished at global step %d", sess.global_step)
    return 0
