#!/bin/bash
# Channel x workgroup limit of the conv prologue finalize, shipped database.
OUT=${1:-gpurun_out/cfinw}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-4} "w19=DRN_TUNE_DB=$DB DRN_CFIN_MAX_WORK=524288" "w18=DRN_TUNE_DB=$DB DRN_CFIN_MAX_WORK=262144" \
  "w20=DRN_TUNE_DB=$DB DRN_CFIN_MAX_WORK=1048576" "never=DRN_TUNE_DB=$DB DRN_CFIN_MAX_WORK=1000000000000" || exit 1
