#!/bin/bash
# Library A/B on one box: the tree's library vs variant libraries (gpu_variants/<name>), CIFAR bs32 /
# bs128 (HIP-graph step) and ResNet-50 bs128, interleaved; one bench.py run per point.
#   ARMS="new gdec nofast" scripts/gpu_ab_libs.sh <outdir>
OUT=${1:-gpurun_out/ablibs}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
ARMS=${ARMS:-"new nofast"}
run() {  # run <label> <lib> <env...> -- <bench args...>
  local label="$1" lib="$2"; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  line=$(env DRN_KERNEL_LIB=$lib "${envs[@]}" timeout -k 10 180 python bench.py --steps ${STEPS:-40} --warmup 5 "$@" 2>>"$OUT/ab.err" | grep '^{') || { echo "[$label] failed"; tail -5 "$OUT/ab.err"; exit 1; }
  echo "$label $line" >> "$OUT/ab.jsonl"
  echo "$label: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms graph", d["config"].get("hip_graph"))')" | tee -a "$OUT/ab.txt"
}
for rep in 1 2; do
  for arm in $ARMS; do
    lib=""; [ $arm != new ] && lib=gpu_variants/$arm/libdrn_kernels.so
    run "$arm cifar bs32" "$lib" X=1 -- --dataset cifar10 --batch_size 32
    run "$arm cifar bs128" "$lib" X=1 -- --dataset cifar10 --batch_size 128
    run "$arm rn50 side192" "$lib" DRN_SIDE_CUS=192 -- --graph 0
  done
done
