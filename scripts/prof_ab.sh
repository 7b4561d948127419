#!/bin/bash
# Kernel traces of one bench step under two environment variants (run on the GPU box):
#   scripts/prof_ab.sh <outdir> "ENV=a" "ENV=b" [...]
# writes <outdir>/v<i>/step_summary.txt per variant; stops at the first failure.
ROOT=$(pwd)
OUT="$1"; shift
export PYTHONPATH=$ROOT
i=0
for v in "$@"; do
  d="$ROOT/$OUT/v$i"; mkdir -p "$d"
  echo "$v" > "$d/variant.txt"
  (cd /tmp && export TMPDIR=/tmp && env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d/prof" -o step \
     --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --graph 0 ${PROF_ARGS:-} > "$d/prof.log" 2>&1) || { echo "variant [$v] failed"; exit 1; }
  python3 scripts/prof_step.py "$d/prof/step_kernel_trace.csv" 0 > "$d/step_summary.txt" || exit 1
  head -1 "$d/step_summary.txt"
  i=$((i+1))
done
