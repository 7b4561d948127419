#!/bin/bash
# Confirmation round of the knob sweep (shipped database in every variant).
OUT=${1:-gpurun_out/sweep2}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-4} "base=DRN_TUNE_DB=$DB" "rep16=DRN_TUNE_DB=$DB DRN_STATS_REPLICAS=16" \
  "fing1k=DRN_TUNE_DB=$DB DRN_BN_FIN_GRID=1024" "both=DRN_TUNE_DB=$DB DRN_STATS_REPLICAS=16 DRN_BN_FIN_GRID=1024" || exit 1
