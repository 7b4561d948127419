#!/bin/bash
# Build the kernel-selection database on the GPU, then A/B the bench with it vs per-run tuning.
OUT=${1:-gpurun_out/db}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
rm -f "$OUT/tune_db.json"
DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json timeout -k 10 900 python -u scripts/make_tune_db.py > "$OUT/make.log" 2>&1 || { tail "$OUT/make.log"; exit 1; }
cat "$OUT/make.log"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "db=DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json" "tune=DRN_TUNE_DB=off" || exit 1
for bs in 128 32; do
  DRN_TUNE_DB=$(pwd)/$OUT/tune_db.json timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/cifar_db.jsonl" 2>> "$OUT/cifar.err" || exit 1
done
cut -c1-200 "$OUT/cifar_db.jsonl"
