#!/bin/bash
# CIFAR: atomic-only weight-gradient split-K (no reduction launches) vs the tuner's choice.
OUT=${1:-gpurun_out/ca}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in tuner atomic; do
    for bs in 128 32; do
      e=""; [ $v = atomic ] && e="DRN_WGRAD_ATOMIC_ONLY=1"
      line=$(env DRN_TUNE_DB=off $e timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 2>> "$OUT/err.txt") || exit 1
      echo "$r $v bs=$bs $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
    done
  done
done
