#!/bin/bash
# Loader iteration on one GPU box: the conv / executor GPU tests, per-layer conv timings and the
# step bench of the tree's library vs the -DDRN_NO_FAST_LOADER variant (same box, interleaved),
# plus workgroup timelines of the weight-gradient kernel.
#   scripts/gpu_wgrad_iter.sh <outdir>
OUT=${1:-gpurun_out/witer}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
if [ "${TESTS:-}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_ops_gpu.py tests/test_executor_gpu.py} \
    -m gpu -x -q --timeout 170 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -2 "$OUT/tests.log"
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; fi
fi
NOFAST=gpu_variants/nofast/libdrn_kernels.so
for arm in new old; do
  lib=""; [ $arm = old ] && lib=$NOFAST
  DRN_KERNEL_LIB=$lib timeout -k 10 300 python -u scripts/kernel_bench.py --iters 20 --no_bn 2>&1 | grep -v amdgpu.ids > "$OUT/kbench_$arm.txt" || { echo "kbench failed"; tail "$OUT/kbench_$arm.txt"; exit 1; }
  tail -1 "$OUT/kbench_$arm.txt"
done
if [ -f gpu_variants/trace/libdrn_kernels.so ]; then
  for spec in "14 1024 256 1 1 2 512" "56 64 256 1 1 2 512" "14 256 256 3 1 2 512"; do
    DRN_KERNEL_LIB=gpu_variants/trace/libdrn_kernels.so timeout -k 10 60 python -u scripts/trace_wgrad.py $spec \
      2>&1 | grep --line-buffered -v amdgpu.ids | tee -a "$OUT/wtrace.txt" || exit 1
  done
fi
for rep in 1 2; do
  for arm in new old; do
    lib=""; [ $arm = old ] && lib=$NOFAST
    line=$(DRN_KERNEL_LIB=$lib timeout -k 10 180 python bench.py --steps 40 --warmup 5 $BENCH_ARGS 2>>"$OUT/bench.err" | grep '^{') || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
    echo "$arm $line" | tee -a "$OUT/bench.txt" | cut -c1-160
  done
done
