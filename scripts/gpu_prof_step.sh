#!/bin/bash
# Kernel-trace profile of the default ResNet-50 step + idle-interval analysis.
OUT=${1:-gpurun_out/prof1}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --graph 0 > "$ROOT/$OUT/prof.log" 2>&1 || { tail "$ROOT/$OUT/prof.log"; exit 1; }
cd "$ROOT"
python3 scripts/step_streams.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/streams.txt" || true
python3 scripts/idle_intervals.py "$OUT/prof/step_kernel_trace.csv" 10 > "$OUT/idle.txt"
head -8 "$OUT/streams.txt"; cat "$OUT/idle.txt"
