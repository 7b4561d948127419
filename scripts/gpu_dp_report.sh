#!/bin/bash
# DP engine after the no-launch report change: tests, then plain vs single-rank DP benches.
OUT=${1:-gpurun_out/dpr}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_p2p_fault_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2 3; do
  a=$(timeout -k 10 200 python bench.py 2>>"$OUT/err.txt" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])') || exit 1
  b=$(DRN_BENCH_DP=1 timeout -k 10 200 python bench.py 2>>"$OUT/err.txt" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])') || exit 1
  echo "$r plain $a dp $b" | tee -a "$OUT/ab.txt"
done
