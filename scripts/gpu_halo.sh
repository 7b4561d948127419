#!/bin/bash
# Halo conv: correctness tests, then the layer benchmark. Stops at the first failure.
OUT=${1:-gpurun_out/halo}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -5 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/halo_bench.py 128 20 > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.jsonl"
