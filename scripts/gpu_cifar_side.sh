#!/bin/bash
# CIFAR graph step with / without the weight-gradient side stream (shipped database).
OUT=${1:-gpurun_out/cs}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for r in 1 2 3; do
  for ws in 1 0; do
    for bs in 128 32; do
      line=$(DRN_WGRAD_STREAM=$ws timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 2>> "$OUT/err.txt") || exit 1
      echo "$r side=$ws bs=$bs $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["hip_graph"])')" | tee -a "$OUT/ab.txt"
    done
  done
done
