#!/bin/bash
# Interleaved A/B of bench.py variants inside ONE GPU call (timings are only compared within
# one box: boxes differ by 1-2 %).
#   scripts/gpu_ab.sh <outdir> <rounds> "<bench args>" name1="VAR=v ..." name2="" ...
# A variant's environment selects e.g. another kernel library (DRN_KERNEL_LIB=ab/libbase.so).
# Prints one "name round ms/step" line per run; the JSON lines land in <outdir>/<name>.jsonl.
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
export PYTHONPATH=$(pwd)
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    env $envs timeout -k 10 400 python3 bench.py $ARGS >> "$OUT/$name.jsonl" 2> "$OUT/$name.$r.err" \
      || { echo "$name round $r failed"; tail -5 "$OUT/$name.$r.err"; exit 1; }
    echo "$name r$r $(tail -1 "$OUT/$name.jsonl" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
