#!/bin/bash
# Vendor-library ceiling per conv shape + the real-training HW-queue audit (CIFAR CLI).
OUT=${1:-gpurun_out/ceil}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u scripts/lib_ceiling.py 128 20 > "$OUT/ceiling.jsonl" 2> "$OUT/ceiling.err" || { tail "$OUT/ceiling.err"; exit 1; }
cat "$OUT/ceiling.jsonl"
[ -n "$NOAUDIT" ] && exit 0
bash scripts/queue_audit.sh "$OUT/queue_audit"
