#!/bin/bash
# A/B sweep of environment knobs on the 1-GPU bench (run from the repo root on the GPU box):
#   scripts/env_sweep.sh <outfile> "ENV1=a ENV2=b" "ENV1=c" ...
# Each variant runs bench.py under its own time limit; the sweep stops at the first failure.
OUT="$1"; shift
mkdir -p "$(dirname "$OUT")"
export PYTHONPATH=$(pwd)
: > "$OUT"
for v in "$@"; do
  line=$(env $v timeout -k 10 120 python bench.py --steps ${SWEEP_STEPS:-40} --warmup 5 ${SWEEP_ARGS:-} 2>>"$OUT.err")
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant [$v] failed rc=$rc" | tee -a "$OUT"; exit $rc; fi
  ms=$(echo "$line" | python -c 'import json,sys; print(json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1])["ms_per_step"])')
  echo "$ms ms  [$v]" | tee -a "$OUT"
done
