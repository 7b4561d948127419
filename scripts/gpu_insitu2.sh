#!/bin/bash
# In-situ re-timing over 4 vs 8 tuner finalists.
OUT=${1:-gpurun_out/insitu2}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "top4=DRN_TUNE_TOP=4" "top8=DRN_TUNE_TOP=8 DRN_PRINT_TUNE=1" || exit 1
grep -h "in-situ" "$OUT/top8.err"
