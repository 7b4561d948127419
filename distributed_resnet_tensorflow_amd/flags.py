"""tf.app.flags-compatible command-line flags (absl is not available here).

Every entry point registers the UNION of the reference's flags so that a flag
defined only in one reference script (e.g. --data_format, missing from the ImageNet scripts:
SURVEY Q3) never crashes another, plus this framework's own flags. Accepted syntaxes match
gflags/absl: ``--flag=value``, ``--flag value``, boolean ``--flag``, ``--noflag`` and
``--flag=True/False/true/false/1/0`` (the reference scripts pass ``--sync_replicas=True``,
scripts/submit_cifar_daint_dist.sh:42; ``--eval_once=True``, scripts/submit_horovod_cifar_eval.sh:11).

    from distributed_resnet_tensorflow_amd import flags
    FLAGS = flags.define_reference_flags(batch_size=128)   # per-entry-point defaults
    argv = FLAGS(sys.argv)                                  # parse
"""
from __future__ import annotations

import sys
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional


class FlagsError(ValueError):
    pass


def _parse_bool(v: str) -> bool:
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n"):
        return False
    raise FlagsError(f"not a boolean: {v!r}")


@dataclass
class _Flag:
    name: str
    default: Any
    help: str
    parse: Callable[[str], Any]
    kind: str
    value: Any = None
    present: bool = False


class FlagValues:
    def __init__(self):
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)

    # -- definition -------------------------------------------------------------------------
    def _define(self, name, default, help_, parse, kind):
        fl = self._flags
        if name in fl:  # re-definition keeps the first definition (module re-imports)
            return
        fl[name] = _Flag(name, default, help_, parse, kind, default)

    def set_default(self, name, value):
        f = self._flags[name]
        f.default = value
        if not f.present:
            f.value = value

    # -- access -------------------------------------------------------------------------------
    def __getattr__(self, name):
        fl = object.__getattribute__(self, "_flags")
        if name in fl:
            return fl[name].value
        raise AttributeError(f"unknown flag --{name}")

    def __setattr__(self, name, value):
        fl = self._flags
        if name not in fl:
            raise AttributeError(f"unknown flag --{name}")
        fl[name].value = value

    def __contains__(self, name):
        return name in self._flags

    def flag_values_dict(self) -> Dict[str, Any]:
        return {k: f.value for k, f in self._flags.items()}

    def is_present(self, name) -> bool:
        return self._flags[name].present

    # -- parsing ------------------------------------------------------------------------------
    def __call__(self, argv: List[str], known_only: bool = False) -> List[str]:
        rest = [argv[0]] if argv else []
        args = list(argv[1:])
        i = 0
        while i < len(args):
            a = args[i]
            i += 1
            if a == "--":
                rest.extend(args[i:])
                break
            if not a.startswith("-") or a == "-":
                rest.append(a)
                continue
            body = a.lstrip("-")
            if "=" in body:
                name, val = body.split("=", 1)
                has_val = True
            else:
                name, val, has_val = body, None, False
            f = self._flags.get(name)
            if f is None and name.startswith("no") and name[2:] in self._flags \
                    and self._flags[name[2:]].kind == "bool" and not has_val:
                f = self._flags[name[2:]]
                f.value, f.present = False, True
                continue
            if f is None:
                if known_only:
                    rest.append(a)
                    continue
                raise FlagsError(f"Unknown command line flag '{name}'")
            if f.kind == "bool":
                if not has_val:
                    # `--flag True` (space separated) is also accepted for bools
                    if i < len(args) and args[i].lower() in ("true", "false", "1", "0"):
                        val = args[i]
                        i += 1
                    else:
                        val = "true"
                f.value = _parse_bool(val)
            else:
                if not has_val:
                    if i >= len(args):
                        raise FlagsError(f"Flag --{name} must have a value")
                    val = args[i]
                    i += 1
                try:
                    f.value = None if (val is None) else f.parse(val)
                except ValueError as e:
                    raise FlagsError(f"Flag --{name}: {e}") from e
            f.present = True
        object.__setattr__(self, "_parsed", True)
        return rest

    def reset(self):
        for f in self._flags.values():
            f.value, f.present = f.default, False

    def help_text(self) -> str:
        lines = []
        for f in sorted(self._flags.values(), key=lambda x: x.name):
            lines.append(f"  --{f.name}: {f.help} (default: {f.default!r})")
        return "\n".join(lines)


FLAGS = FlagValues()


def _none_or(parse):
    def p(v):
        if v is None or str(v) in ("None", ""):
            return None
        return parse(v)
    return p


def DEFINE_string(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, lambda v: v if v != "None" else None, "string")


def DEFINE_integer(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, _none_or(int), "int")


def DEFINE_float(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, _none_or(float), "float")


def DEFINE_bool(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, _parse_bool, "bool")


DEFINE_boolean = DEFINE_bool


def define_reference_flags(flag_values: FlagValues = FLAGS, **defaults) -> FlagValues:
    """Registers the union flag set; keyword args override per-entry-point defaults."""
    fv = flag_values
    S, I, Fl, B = DEFINE_string, DEFINE_integer, DEFINE_float, DEFINE_bool
    # ---- reference flags (resnet_cifar_main.py:32-86, resnet_imagenet_main.py:33-81, eval :28-55) ----
    S("dataset", "cifar10", "cifar10, cifar100 or imagenet.", fv)
    S("mode", "train", "train or eval.", fv)
    S("train_data_path", "", "Filepattern / directory for training data.", fv)
    S("eval_data_path", "", "Filepattern / directory for eval data.", fv)
    I("image_size", 32, "Image side length.", fv)
    S("train_dir", "", "Directory to keep training outputs.", fv)
    S("eval_dir", "", "Directory to keep eval outputs.", fv)
    I("eval_batch_count", 50, "Number of batches to eval.", fv)
    B("eval_once", False, "Whether evaluate the model only once.", fv)
    S("log_root", "", "Directory to keep the checkpoints.", fv)
    I("num_gpus", 0, "Number of gpus used for training (0 = CPU).", fv)
    I("task_index", None, "Worker task index, should be >= 0. task_index=0 is the chief.", fv)
    I("replicas_to_aggregate", None, "Accepted for compatibility; all replicas are aggregated.", fv)
    I("train_steps", 2000, "Number of (global) training steps to perform.", fv)
    I("num_epochs", 90, "Number of training epochs (ImageNet input repeat).", fv)
    I("batch_size", 32, "Per-worker training batch size.", fv)
    Fl("learning_rate", 0.01, "Learning rate (LRNet/Adam only, as in the reference).", fv)
    B("sync_replicas", False, "Synchronous replicas (all-reduce average every step); False with "
      "--job_name set = 1-step-delayed all-reduce (async-PS analog).", fv)
    B("existing_servers", False, "Accepted for compatibility (no in-process gRPC servers here).", fv)
    S("ps_hosts", "localhost:2222", "Comma-separated list of hostname:port pairs (PS tasks exit).", fv)
    S("worker_hosts", "localhost:2223,localhost:2224", "Comma-separated list of hostname:port pairs.", fv)
    S("job_name", None, "job name: worker or ps (None = serial / launcher-provided rank).", fv)
    S("data_format", "channels_first", "Accepted; the MI355X kernels are NHWC (channels_last) natively.", fv)
    I("num_intra_threads", 0, "CPU intra-op threads (torch.set_num_threads) when > 0.", fv)
    I("num_inter_threads", 0, "CPU inter-op threads (torch.set_num_interop_threads) when > 0.", fv)
    B("use_horovod", False, "All-reduce data parallelism (default engine; Horovod analog).", fv)
    I("hidden_units", 100, "LRNet hidden units.", fv)
    # ---- framework flags ----
    I("resnet_size", None, "ResNet depth (reference hard-codes 50): CIFAR 6n+2, ImageNet 18..200.", fv)
    S("model", "resnet", "resnet | wide_resnet | lrnet.", fv)
    I("width_multiplier", 2, "Bottleneck width multiplier for --model=wide_resnet (WRN-50-2).", fv)
    S("precision", "bf16", "Compute precision of the GPU path (bf16 activations, fp32 master).", fv)
    B("synthetic_data", False, "Use synthetic data of the dataset's shape (benchmarks).", fv)
    I("save_checkpoint_secs", 60, "Checkpoint period in seconds (reference: 60).", fv)
    I("save_summaries_steps", 100, "Summary period in steps (reference: 100).", fv)
    I("log_every_n_steps", 20, "Logging period in steps (CIFAR 20, ImageNet 40).", fv)
    I("max_to_keep", 5, "Checkpoints kept in log_root (TF Saver default 5).", fv)
    S("profile_steps", "", "a:b -> roctx-mark and torch-profile steps a..b.", fv)
    S("allreduce", "rccl", "Gradient all-reduce: rccl (RCCL ring/tree over xGMI; gloo on CPU), p2p (one-shot "
      "HIP-IPC peer kernel, one node), auto (p2p when the gradient is <= 64 MB).", fv)
    S("allreduce_wire", "fp32", "Gradient dtype on the wire: fp32, or bf16 (half the all-reduce bytes, fp32 "
      "accumulation in the P2P kernel; the Horovod fp16-compression analog).", fv)
    Fl("bucket_mb", 25.0, "Gradient all-reduce bucket size cap (MB of fp32).", fv)
    B("optimizer_sharding", False, "ZeRO-1-style sharded optimizer (the parameter-server sharding analog, "
      "SURVEY P3): reduce-scatter the gradient buckets, update 1/N of the weights and momentum per rank, "
      "all-gather the bf16 compute weights.", fv)
    I("collective_timeout_secs", 600, "Process-group timeout and collective-watchdog limit: a rank whose "
      "gradient exchange stalls this long exits (the launcher restarts the job from its checkpoint).", fv)
    I("fault_inject_step", -1, "Kill this process at the given global step (fault-injection tests).", fv)
    I("fault_inject_rank", 0, "Rank that --fault_inject_step applies to.", fv)
    B("hip_graph", True, "Capture the single-GPU training step in a HIP graph.", fv)
    I("seed", 0, "Random seed (weights, data order, augmentation).", fv)
    Fl("lr_schedule_scale", 1.0, "Scale of every step boundary of the reference LR schedule (1.0 = the "
       "reference; e.g. 0.05 decays the CIFAR LR at 2k/3k/4k steps for short runs).", fv)
    I("eval_interval_secs", 60, "Eval poller period (reference sleeps 60 s).", fv)
    Fl("weight_decay", None, "Override the dataset's weight decay (CIFAR 2e-4, ImageNet 1e-4).", fv)
    I("num_workers", 2, "Host data-loader worker threads.", fv)
    S("input_workers", "process", "ImageNet JPEG decode workers: process (spawned decode processes, scales with "
      "cores) or thread (a thread pool; JPEG decode partly holds the GIL).", fv)
    S("master_addr", "", "Rendezvous address override (default MASTER_ADDR or worker_hosts[0]).", fv)
    for k, v in defaults.items():
        fv.set_default(k, v)
    return fv


def parse(argv: Optional[List[str]] = None, flag_values: FlagValues = FLAGS) -> List[str]:
    return flag_values(list(sys.argv if argv is None else argv))
