"""Learning-rate schedules of the reference `_LearningRateSetterHook`s.

The reference feeds `lrn_rate` each step from the global step of the PREVIOUS run() call
(after_run sets the value used by the next before_run; begin() seeds the first step).
"""
from __future__ import annotations


def cifar_lr(step: int) -> float:
    """resnet_cifar_main.py:287-307: 0.1 -> 0.01 @40k -> 0.001 @60k -> 1e-4 @80k."""
    if step < 40000:
        return 0.1
    if step < 60000:
        return 0.01
    if step < 80000:
        return 0.001
    return 0.0001


def imagenet_lr(step: int) -> float:
    """resnet_imagenet_main.py:223-247 ("Intel-Caffe 8-node" schedule): linear warm-up
    0.1 -> 0.4 over 6,240 steps, 0.4 until 37,440, 0.04 until 74,880, 0.004 until 99,840,
    then 0.0004."""
    if step < 6240:
        return 0.1 + (0.4 - 0.1) * step / 6240.0
    if step < 37440:
        return 0.4
    if step < 74880:
        return 0.04
    if step < 99840:
        return 0.004
    return 0.0004


class LRSchedule:
    """Mirrors the hook protocol: the LR used for a step is computed from the global step
    returned by the previous step; the very first step uses `first` (CIFAR begin() = 0.1,
    ImageNet begin() = 0.4, resnet_imagenet_main.py:226-227)."""

    def __init__(self, fn, first: float):
        self.fn = fn
        self.next_lr = first

    def lr_for_step(self) -> float:
        return self.next_lr

    def after_step(self, global_step: int):
        self.next_lr = self.fn(global_step)


def for_dataset(dataset: str, step_scale: float = 1.0) -> LRSchedule:
    """The reference's schedule for `dataset`. step_scale (--lr_schedule_scale, an extension for
    short runs: tests, smoke trainings) stretches / compresses every step boundary: 0.05 puts
    the CIFAR decays at 2k / 3k / 4k steps instead of 40k / 60k / 80k. 1.0 = the reference."""
    if step_scale <= 0:
        raise ValueError(f"--lr_schedule_scale must be > 0, got {step_scale}")
    base = imagenet_lr if dataset == "imagenet" else cifar_lr
    fn = base if step_scale == 1.0 else (lambda step: base(int(step / step_scale)))
    return LRSchedule(fn, 0.4 if dataset == "imagenet" else 0.1)
