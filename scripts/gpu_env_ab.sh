#!/bin/bash
# Interleaved A/B of bench.py under environment variants (each variant re-tunes: DRN_TUNE_DB=off).
#   scripts/gpu_env_ab.sh <outdir> <rounds> "<name>=<env assignments>" ...
OUT=$1; ROUNDS=$2; shift 2
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    line=$(env DRN_TUNE_DB=off $envs timeout -k 10 300 python bench.py 2>> "$OUT/$name.err") || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    ms=$(echo "$line" | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$r $name $ms" | tee -a "$OUT/ab.txt"
  done
done
