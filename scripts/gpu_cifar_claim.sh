#!/bin/bash
# CIFAR + ResNet-50 benches after the claim-span cap (shipped database).
OUT=${1:-gpurun_out/cc}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for i in 1 2; do
  for bs in 128 32; do
    timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/cifar.jsonl" 2>> "$OUT/err.txt" || exit 1
  done
  timeout -k 10 200 python bench.py >> "$OUT/rn50.jsonl" 2>> "$OUT/err.txt" || exit 1
done
python3 -c "
import json
for f in ('$OUT/cifar.jsonl', '$OUT/rn50.jsonl'):
    for l in open(f): d=json.loads(l); print(d['config']['model'], d['config']['global_batch'], d['ms_per_step'])"
