#!/bin/bash
# Full validation on one GPU box: every GPU test, then smoke + benches + a profiled step.
OUT=${1:-gpurun_out/val}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1
rc=$?; tail -3 "$OUT/tests.txt"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.txt" | head -20; exit $rc; }
bash scripts/gpu_r4_base.sh "$OUT"
