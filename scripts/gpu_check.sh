#!/bin/bash
# GPU test suite, then (only if it passed) bench + profile. Stops at the first failure.
OUT=${1:-gpurun_out/pc}
export PYTHONPATH=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/gputests.log
if [ $rc -ne 0 ]; then echo "gpu tests failed rc=$rc"; exit $rc; fi
scripts/gpu_prof.sh "$OUT"
