#!/bin/bash
# ResNet-50 step: HIP-graph replay vs eager (shipped database), after the coarse claims.
OUT=${1:-gpurun_out/gab}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
for r in 1 2; do
  for g in 0 1; do
    line=$(timeout -k 10 300 python bench.py --graph $g 2>> "$OUT/err.txt") || { tail "$OUT/err.txt"; exit 1; }
    echo "$r graph=$g $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
  done
done
