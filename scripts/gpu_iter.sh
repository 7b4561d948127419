#!/bin/bash
# One GPU iteration on a fresh box: selected GPU tests, the ResNet-50 conv config sweep, the
# bench + kernel-trace profile, optional extra probes. Stops at the first failure.
#   TESTS="tests/test_x.py ..." K="pytest -k expression" SWEEP=1 BENCH=1 PROBE="cmd" scripts/gpu_iter.sh <outdir>
OUT=${1:-gpurun_out/iter}
TESTS=${TESTS:-"tests/test_ops_gpu.py"}
K=${K:-""}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 170 --timeout-method thread \
    ${K:+-k "$K"} > "$OUT/tests.log" 2>&1
  rc=$?
  tail -3 "$OUT/tests.log"
  if [ $rc -ne 0 ]; then echo "gpu tests failed rc=$rc"; grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; fi
fi
if [ "${SWEEP:-1}" = "1" ]; then
  bash scripts/sweep_rn50.sh > "$OUT/sweep.txt" 2>&1 || { echo "sweep failed"; tail "$OUT/sweep.txt"; exit 1; }
  grep -v amdgpu.ids "$OUT/sweep.txt"
fi
if [ "${BENCH:-1}" = "1" ]; then
  bash scripts/gpu_prof.sh "$OUT" || exit 1
fi
if [ -n "$PROBE" ]; then
  bash -c "$PROBE" > "$OUT/probe.log" 2>&1
  rc=$?
  tail -20 "$OUT/probe.log"
  exit $rc
fi
