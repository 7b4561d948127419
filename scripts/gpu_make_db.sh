#!/bin/bash
# Build the kernel-selection database on the GPU (scripts/make_tune_db.py: the benchmark
# configurations with the thorough tuner), then bench with it. Run from the repo root; copy
# <outdir>/tune_db.json to distributed_resnet_tensorflow_amd/ops/tune_db.json to ship it.
#   scripts/gpu_make_db.sh <outdir>
OUT=${1:-gpurun_out/db}
export PYTHONPATH=$(pwd)
# the shipped database is neither consulted nor merged: the new file is the complete section, and
# the follow-up benches measure its choices
export DRN_TUNE_DB_SYSTEM=off
mkdir -p "$OUT"
rm -f "$OUT/tune_db.json"
DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json timeout -k 10 900 python -u scripts/make_tune_db.py > "$OUT/make.log" 2>&1 || { tail "$OUT/make.log"; exit 1; }
cat "$OUT/make.log"
for i in 1 2; do
  DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json timeout -k 10 200 python bench.py >> "$OUT/bench_rn50.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
done
for bs in 128 32; do
  DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench_cifar.jsonl" 2>> "$OUT/bench.err" || exit 1
done
cut -c1-200 "$OUT"/bench_*.jsonl
