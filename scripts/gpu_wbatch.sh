#!/bin/bash
# Weight gradients per side-stream wait: tests, then step A/B with the shipped database.
OUT=${1:-gpurun_out/wb}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
DRN_WGRAD_BATCH=3 timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "b1=DRN_TUNE_DB=$DB DRN_WGRAD_BATCH=1" "b2=DRN_TUNE_DB=$DB DRN_WGRAD_BATCH=2" \
  "b4=DRN_TUNE_DB=$DB DRN_WGRAD_BATCH=4" || exit 1
