#!/bin/bash
# Every conv kernel configuration on the ResNet-50 v2 bs128 forward / data-gradient shapes with
# the epilogue flags the training step uses (scripts/cfg_sweep.py prints the 12 fastest per shape).
#   scripts/sweep_rn50.sh > gpurun_out/sweep.txt
export PYTHONPATH=$(pwd)
run() { timeout -k 10 120 python scripts/cfg_sweep.py "$@" || exit 1; }
# forward
run 128 56 64 64 1 1 pro stats
run 128 56 64 64 3 1 stats
run 128 56 64 256 1 1 pro res stats
run 128 56 256 64 1 1 pro stats
run 128 56 256 128 1 1 pro stats
run 128 56 128 128 3 2 stats
run 128 28 128 128 3 1 stats
run 128 28 128 512 1 1 pro res stats
run 128 28 512 128 1 1 pro stats
run 128 14 256 256 3 1 stats
run 128 14 256 1024 1 1 pro res stats
run 128 14 1024 256 1 1 pro stats
run 128 7 512 512 3 1 pro stats
run 128 7 512 2048 1 1 pro res stats
run 128 7 2048 512 1 1 pro stats
# data gradients (channels swapped; the 3x3 ones are stride-1 convs of dY with flipped weights)
run 128 56 256 64 1 1 stats
run 128 28 512 128 1 1 stats
run 128 14 1024 256 1 1 stats
run 128 7 2048 512 1 1 stats
run 128 7 512 2048 1 1 res stats
