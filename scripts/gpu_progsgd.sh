#!/bin/bash
# Overlapped per-block optimizer: tests, then step A/B (per-run tuning in both variants).
OUT=${1:-gpurun_out/prog}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "noprog=DRN_PROG_SGD=0" "prog=DRN_PROG_SGD=1" "prog_g1024=DRN_PROG_SGD=1 DRN_SGD_GRID=1024" || exit 1
