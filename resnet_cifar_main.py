#!/usr/bin/env python3
"""resnet_cifar_main.py — same entry point, flags and behaviour as the reference's resnet_cifar_main.py, running on
the MI355X-native engine (see distributed_resnet_tensorflow_amd/cli.py for the mapping)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_resnet_tensorflow_amd.cli import cifar_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(cifar_main())
