#!/bin/bash
# In-situ re-timing of the conv tuner's finalists: step A/B and how many choices it changes.
OUT=${1:-gpurun_out/insitu}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "iso=DRN_INSITU_TUNE=0" "insitu=DRN_INSITU_TUNE=1 DRN_PRINT_TUNE=1" || exit 1
grep -h "in-situ" "$OUT/insitu.err"
