#!/bin/bash
# BN apply unroll: tests, then step A/B of the consumer-finalize grid limit.
OUT=${1:-gpurun_out/bnu}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_executor_gpu.py -x -q --timeout 300 \
  --timeout-method thread -k "bn or finalize or executor or pool" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "def=DRN_CFIN_MAX_BLOCKS=2048" "cfin8k=DRN_CFIN_MAX_BLOCKS=8192" || exit 1
