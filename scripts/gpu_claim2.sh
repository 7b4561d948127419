#!/bin/bash
# Gradient-buffer claims: wait span after the reader (0 = one wait per claim), shipped database.
OUT=${1:-gpurun_out/claim2}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "span0=DRN_TUNE_DB=$DB DRN_CLAIM_SPAN=0" "span6=DRN_TUNE_DB=$DB DRN_CLAIM_SPAN=6" \
  "span12=DRN_TUNE_DB=$DB DRN_CLAIM_SPAN=12" "span24=DRN_TUNE_DB=$DB DRN_CLAIM_SPAN=24" || exit 1
