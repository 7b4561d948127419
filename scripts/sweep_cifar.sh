#!/bin/bash
# Conv configurations on the CIFAR ResNet-50 (6n+2) stage-1 shapes (K = 16 outputs: 1x1 64->16
# reduce, 3x3 16->16, and the data gradients that produce 16 channels) at batch 128 and 32.
#   scripts/sweep_cifar.sh > gpurun_out/sweep_cifar.txt
export PYTHONPATH=$(pwd)
run() { timeout -k 10 120 python scripts/cfg_sweep.py "$@" || exit 1; }
for n in 128 32; do
  run $n 32 64 16 1 1 pro stats
  run $n 32 16 16 3 1 pro stats
  run $n 32 64 16 1 1 stats
  run $n 32 16 16 3 1 stats
  run $n 16 128 32 1 1 pro stats
  run $n 16 32 32 3 1 pro stats
done
