#!/bin/bash
# Coarse gradient-buffer claims: step A/B over the claim lag, with the shipped kernel database.
OUT=${1:-gpurun_out/claim}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "lag0=DRN_TUNE_DB=$DB DRN_CLAIM_LAG=0" "lag6=DRN_TUNE_DB=$DB DRN_CLAIM_LAG=6" \
  "lag12=DRN_TUNE_DB=$DB DRN_CLAIM_LAG=12" || exit 1
