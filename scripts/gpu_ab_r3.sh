#!/bin/bash
# Step-mode / side-stream A/B on one GPU (ResNet-50 bs128 unless noted), then a CIFAR bs32 kernel
# profile. Each variant is its own bench.py run under its own time limit; stops at the first failure.
#   scripts/gpu_ab_r3.sh <outdir>
OUT=${1:-gpurun_out/ab}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
run() {  # run <label> <env...> -- <bench args...>
  local label="$1"; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  line=$(env "${envs[@]}" timeout -k 10 180 python bench.py --steps 40 --warmup 5 "$@" 2>>"$OUT/ab.err" | grep '^{') || { echo "[$label] failed"; tail -5 "$OUT/ab.err"; exit 1; }
  echo "$line" >> "$OUT/ab.jsonl"
  echo "$label: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", d["config"].get("hip_graph"))')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2; do
  run "auto" X=1 --
  run "eager+prio" X=1 -- --graph 0
  run "graph" X=1 -- --graph 1
  run "eager+prio side224" DRN_SIDE_CUS=224 -- --graph 0
  run "eager+prio side192" DRN_SIDE_CUS=192 -- --graph 0
done
for bs in 128 32; do
  run "cifar bs$bs auto" X=1 -- --dataset cifar10 --batch_size $bs
done
bash scripts/gpu_prof.sh "$OUT/cifar32" --dataset cifar10 --batch_size 32 > /dev/null 2>&1 || { echo "cifar prof failed"; exit 1; }
head -1 "$OUT/cifar32/step_summary.txt"
