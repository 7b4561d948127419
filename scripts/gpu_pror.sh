#!/bin/bash
# Register-side BN prologue (PROR): correctness, then step A/B against the LDS rewrite.
OUT=${1:-gpurun_out/pror}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_geometry_gpu.py -x -q --timeout 500 \
  --timeout-method thread -k "glds_configs or prologue or splitk or bench_geometry" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-3} "lds=DRN_PRO_REG=0" "reg=DRN_PRO_REG=1" || exit 1
