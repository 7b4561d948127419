#!/bin/bash
# Step-mode / side-stream A/B on one GPU (ResNet-50 bs128 unless noted), for the tree's library
# ("new") and the -DDRN_NO_FAST_LOADER variant ("old"), interleaved on one box; then CIFAR benches
# and a CIFAR bs32 kernel profile. Each variant is its own bench.py run under its own time limit;
# stops at the first failure.
#   scripts/gpu_ab_r3.sh <outdir>
OUT=${1:-gpurun_out/ab}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
NOFAST=gpu_variants/nofast/libdrn_kernels.so
run() {  # run <label> <env...> -- <bench args...>
  local label="$1"; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  line=$(env "${envs[@]}" timeout -k 10 180 python bench.py --steps 40 --warmup 5 "$@" 2>>"$OUT/ab.err" | grep '^{') || { echo "[$label] failed"; tail -5 "$OUT/ab.err"; exit 1; }
  echo "$label $line" >> "$OUT/ab.jsonl"
  echo "$label: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms graph", d["config"].get("hip_graph"))')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2; do
  for arm in new old; do
    lib=""; [ $arm = old ] && lib=$NOFAST
    run "$arm auto" DRN_KERNEL_LIB=$lib --
    run "$arm eager+prio side192" DRN_KERNEL_LIB=$lib DRN_SIDE_CUS=192 -- --graph 0
    run "$arm eager+prio side160" DRN_KERNEL_LIB=$lib DRN_SIDE_CUS=160 -- --graph 0
  done
done
for bs in 128 32; do
  for arm in new old; do
    lib=""; [ $arm = old ] && lib=$NOFAST
    run "$arm cifar bs$bs" DRN_KERNEL_LIB=$lib -- --dataset cifar10 --batch_size $bs
  done
done
if [ -n "$CPROF" ]; then
  bash scripts/gpu_prof.sh "$OUT/cifar32" --dataset cifar10 --batch_size 32 > /dev/null 2>&1 || { echo "cifar prof failed"; exit 1; }
  head -1 "$OUT/cifar32/step_summary.txt"
fi
if [ -n "$QAUDIT" ]; then
  timeout -k 10 700 bash scripts/queue_audit.sh "$OUT/queue" > "$OUT/queue_audit.txt" 2>&1 || { echo "queue audit failed"; tail -20 "$OUT/queue_audit.txt"; exit 1; }
  grep -E "==|stream|concurrently|gaps" "$OUT/queue_audit.txt" | head -30
fi
