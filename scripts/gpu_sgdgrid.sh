#!/bin/bash
# Optimizer grid cap vs the stem weight-gradient tail (per-run tuning in every variant).
OUT=${1:-gpurun_out/sgdg}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "g8192=DRN_SGD_GRID=8192" "g2048=DRN_SGD_GRID=2048" "g1024=DRN_SGD_GRID=1024" || exit 1
