#!/bin/bash
# Diagnostics pass on one GPU box (each step time-limited, stops at the first failure):
# isolated per-layer conv timings, per-workgroup conv timelines (trace variant library), the
# CIFAR eval probe, the P2P failure tests and the HW-queue audit.
#   scripts/gpu_diag.sh <outdir>
OUT=${1:-gpurun_out/diag}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
set -o pipefail
if [ -n "$KBENCH" ]; then
  echo "== kernel_bench"
  timeout -k 10 300 python -u scripts/kernel_bench.py --iters 10 --pro --no_bn --json "$OUT/kernel_bench.json" \
    > "$OUT/kernel_bench.txt" 2>&1 || { tail "$OUT/kernel_bench.txt"; exit 1; }
  tail -25 "$OUT/kernel_bench.txt"
fi
if [ -n "$ENVAB" ]; then
  echo "== env A/B (eager steps)"
  SWEEP_ARGS="--graph 0" timeout -k 10 600 bash scripts/env_sweep.sh "$OUT/env_ab.txt" $ENVAB || exit 1
fi
echo "== conv timelines"
if [ -f gpu_variants/trace/libdrn_kernels.so ]; then
  for spec in ${TRACES:-"14 256 256 3 1 0 stats" "14 256 256 3 1 31 stats" "14 256 256 3 1 25 stats" "14 256 256 3 1 33 stats" \
              "14 256 256 3 1 8 stats" "14 256 256 3 1 34 stats"}; do
    DRN_KERNEL_LIB=gpu_variants/trace/libdrn_kernels.so timeout -k 10 60 python -u scripts/trace_conv.py $spec \
      2>&1 | grep --line-buffered -v amdgpu.ids | tee -a "$OUT/timelines.txt" || exit 1
  done
fi
if [ -n "$PROBES" ]; then
  echo "== cifar eval probe"
  timeout -k 10 500 bash scripts/probes/cifar_eval_probe.sh "$OUT/cifar" 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/cifar_probe.txt" || exit 1
  echo "== ImageNet host input rate (this box's CPUs)"
  timeout -k 10 300 python -u scripts/imagenet_input_bench.py --images 2048 --threads 4,8,16 --workers thread,process \
    2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/imagenet_input.txt" || exit 1
  echo "== queue audit"
  timeout -k 10 400 bash scripts/queue_audit.sh "$OUT/queue" 2>&1 | grep --line-buffered -v amdgpu.ids | tee "$OUT/queue_audit.txt" || exit 1
  echo "== p2p failure tests"
  timeout -k 10 400 python -u -m pytest tests/test_p2p_fault_gpu.py -v -x --timeout 170 --timeout-method thread \
    > "$OUT/p2p_fault.log" 2>&1
  rc=$?
  tail -30 "$OUT/p2p_fault.log"
  exit $rc
fi
