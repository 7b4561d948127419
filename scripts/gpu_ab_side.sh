#!/bin/bash
# ResNet-50 bs128 step mode A/B on one box: auto (eager/graph by timing, normal-priority main
# stream) vs eager with the high-priority main stream, with and without a CU-masked weight-
# gradient side stream (DRN_SIDE_CUS), interleaved.
#   scripts/gpu_ab_side.sh <outdir>
OUT=${1:-gpurun_out/abside}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
run() {  # run <label> <env...> -- <bench args...>
  local label="$1"; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  line=$(env "${envs[@]}" timeout -k 10 180 python bench.py --steps 60 --warmup 5 "$@" 2>>"$OUT/ab.err" | grep '^{') || { echo "[$label] failed"; tail -5 "$OUT/ab.err"; exit 1; }
  echo "$label $line" >> "$OUT/ab.jsonl"
  echo "$label: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms graph", d["config"].get("hip_graph"))')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2 3; do
  run "auto" X=1 --
  run "eager+prio" X=1 -- --graph 0
  run "eager+prio side192" DRN_SIDE_CUS=192 -- --graph 0
  run "eager+prio side128" DRN_SIDE_CUS=128 -- --graph 0
  run "eager side192" DRN_SIDE_CUS=192 DRN_MAIN_PRIORITY=0 -- --graph 0
done
