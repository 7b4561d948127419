#!/usr/bin/env python3
"""logist_model.py — the reference's LRNet MLP baseline (logist_model.py:14-86) as an importable
module; train it with `resnet_cifar_main.py --model=lrnet` (the reference never wired it in)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_resnet_tensorflow_amd.models.lrnet import LRNet, train_lrnet  # noqa: E402,F401
