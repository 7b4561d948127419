#!/bin/bash
# Kernel-trace profile of the default (eager) ResNet-50 step: per-kernel step summary, stream
# timeline (main-stream gaps, truly idle GPU). Run from the repo root on the GPU box:
#   scripts/gpu_prof_step.sh <outdir> [bench args...]
OUT=${1:-gpurun_out/prof}; shift
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --graph 0 --plan 0 "$@" > "$ROOT/$OUT/prof.log" 2>&1 || { tail "$ROOT/$OUT/prof.log"; exit 1; }
cd "$ROOT"
python3 scripts/prof_step.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/step_summary.txt"
python3 scripts/step_streams.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/streams.txt" || true
python3 scripts/idle_intervals.py "$OUT/prof/step_kernel_trace.csv" 10 > "$OUT/idle.txt" || true
head -3 "$OUT/step_summary.txt"; head -8 "$OUT/streams.txt"
