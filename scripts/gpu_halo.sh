#!/bin/bash
# Halo conv: correctness tests, the layer benchmark, then the ResNet-50 step bench and the
# bench-geometry correctness test. Stops at the first failure.
OUT=${1:-gpurun_out/halo}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/halo_bench.py 128 20 > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.jsonl"
[ -n "$NOSTEP" ] && exit 0
for i in 1 2; do
  for pol in halo 1x1; do
    echo -n "$pol " >> "$OUT/step.jsonl"
    DRN_BN_MATERIALIZE=$pol DRN_PRINT_TUNE=1 timeout -k 10 300 python bench.py >> "$OUT/step.jsonl" 2>> "$OUT/step_$pol.err" || { tail "$OUT/step_$pol.err"; exit 1; }
  done
done
cut -c1-140 "$OUT/step.jsonl"
grep -c "> (30[0-9]," "$OUT/step_halo.err" || true
timeout -k 10 600 python -u -m pytest tests/test_bench_geometry_gpu.py -x -q --timeout 500 --timeout-method thread > "$OUT/geom.log" 2>&1
rc=$?; tail -3 "$OUT/geom.log"; exit $rc
