#!/bin/bash
# Non-stem optimizer on its own normal-priority stream: tests, then step A/B (shipped database).
OUT=${1:-gpurun_out/opt}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_session_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-4} "main=DRN_TUNE_DB=$DB DRN_OPT_STREAM=0" "opt=DRN_TUNE_DB=$DB DRN_OPT_STREAM=1" || exit 1
