#!/bin/bash
# Data-parallel machinery on one GPU: DP tests, then bench of the single-rank RCCL engine eager vs
# per-segment graphs vs the plain one-GPU graph. Stops at the first failure.
export PYTHONPATH=$(pwd)
O=${1:-gpurun_out/dp}
mkdir -p "$O"
timeout -k 10 300 python -m pytest tests/test_dp_gpu.py -x -q > "$O/tests.log" 2>&1; rc=$?
tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for mode in "0" "1"; do
  DRN_BENCH_DP=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph $mode > "$O/bench_dp_graph$mode.json" 2> "$O/bench_dp_graph$mode.err"; rc=$?
  cat "$O/bench_dp_graph$mode.json"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > "$O/bench_1gpu.json" 2> "$O/bench_1gpu.err"; rc=$?
cat "$O/bench_1gpu.json"; exit $rc
