#!/bin/bash
# Bench + per-kernel profile of the flagship step on one GPU (run from the repo root on the box):
#   scripts/gpu_prof.sh <outdir> [bench args...]
set -e
ROOT=$(pwd)
OUT="$1"; shift
mkdir -p "$ROOT/$OUT"
export PYTHONPATH=$ROOT
timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --graph 0 "$@" > "$ROOT/$OUT/prof.log" 2>&1
cd "$ROOT"
python3 scripts/prof_step.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/step_summary.txt"
python3 scripts/step_streams.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/streams.txt" || true
cat "$OUT/bench.json"
sed -n '/per family/,$p' "$OUT/step_summary.txt" | head -30
grep -E "step wall|stream|gaps|covered|concurrently" "$OUT/streams.txt" || true
