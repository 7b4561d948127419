#!/bin/bash
# CIFAR gradient-buffer pool size (graph step, shipped database).
OUT=${1:-gpurun_out/cb}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
for r in 1 2 3; do
  for nb in 6 12 32; do
    for bs in 128 32; do
      line=$(DRN_GRAD_BUFS=$nb timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 2>> "$OUT/err.txt") || exit 1
      echo "$r bufs=$nb bs=$bs $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
    done
  done
done
