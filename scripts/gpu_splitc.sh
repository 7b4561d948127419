#!/bin/bash
# Channel threshold of the split (separate-launch) BN finalize, shipped database.
OUT=${1:-gpurun_out/splitc}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-4} "c512=DRN_TUNE_DB=$DB DRN_BN_FIN_SPLIT_C=512" "c1024=DRN_TUNE_DB=$DB DRN_BN_FIN_SPLIT_C=1024" \
  "c2048=DRN_TUNE_DB=$DB DRN_BN_FIN_SPLIT_C=2048" "never=DRN_TUNE_DB=$DB DRN_BN_FIN_SPLIT_C=100000" || exit 1
