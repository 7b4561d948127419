#!/bin/bash
# Round-3 status pass on one GPU box: full GPU suite, ResNet-50 bench + kernel-trace profile,
# CIFAR bench at bs 128 / 32. Stops at the first failure.
#   scripts/gpu_round3.sh <outdir>
OUT=${1:-gpurun_out/r3}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=5 -q --timeout 170 --timeout-method thread \
  > "$OUT/gputests.log" 2>&1
rc=$?
tail -3 "$OUT/gputests.log"
if [ $rc -ne 0 ]; then echo "gpu tests failed rc=$rc"; grep -E "Error|assert|FAILED" "$OUT/gputests.log" | head -20; exit $rc; fi
bash scripts/gpu_prof.sh "$OUT" || exit 1
for bs in 128 32; do
  timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 \
    >> "$OUT/cifar_bench.jsonl" 2>> "$OUT/cifar_bench.err" || { tail "$OUT/cifar_bench.err"; exit 1; }
done
cat "$OUT/cifar_bench.jsonl"
if [ -f gpu_variants/trace/libdrn_kernels.so ] && [ -n "$WTRACE" ]; then
  for spec in "14 1024 256 1 1 2 512" "14 1024 256 1 1 6 512" "14 256 256 3 1 2 512" "56 64 64 3 1 2 512" "28 128 512 1 1 2 512"; do
    DRN_KERNEL_LIB=gpu_variants/trace/libdrn_kernels.so timeout -k 10 60 python -u scripts/trace_wgrad.py $spec \
      2>&1 | grep --line-buffered -v amdgpu.ids | tee -a "$OUT/wtrace.txt" || exit 1
  done
fi
