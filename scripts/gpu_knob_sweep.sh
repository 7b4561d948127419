#!/bin/bash
# Env-knob sweep of the current default (shipped database in every variant).
OUT=${1:-gpurun_out/sweep}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "base=DRN_TUNE_DB=$DB" "cfin4k=DRN_TUNE_DB=$DB DRN_CFIN_MAX_BLOCKS=4096" \
  "rep4=DRN_TUNE_DB=$DB DRN_STATS_REPLICAS=4" "rep16=DRN_TUNE_DB=$DB DRN_STATS_REPLICAS=16" \
  "fing1k=DRN_TUNE_DB=$DB DRN_BN_FIN_GRID=1024" "fing4k=DRN_TUNE_DB=$DB DRN_BN_FIN_GRID=4096" \
  "appg4k=DRN_TUNE_DB=$DB DRN_BN_APPLY_GRID=4096" || exit 1
