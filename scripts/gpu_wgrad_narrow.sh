#!/bin/bash
# Narrow-output weight gradient: kernel tests, then CIFAR benches (bs 128 / 32, graph) and a
# CIFAR bs32 step profile. Stops at the first failure.
OUT=${1:-gpurun_out/wn}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
for i in 1 2; do
  for bs in 128 32; do
    timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/cifar.jsonl" 2>> "$OUT/cifar.err" || { tail "$OUT/cifar.err"; exit 1; }
  done
done
cut -c1-200 "$OUT/cifar.jsonl"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset cifar10 --batch_size 32 --steps 5 --warmup 2 --graph 0 > "$ROOT/$OUT/prof.log" 2>&1 || { tail "$ROOT/$OUT/prof.log"; exit 1; }
cd "$ROOT"
python3 scripts/prof_step.py "$OUT/prof/step_kernel_trace.csv" 1000 > "$OUT/step_summary.txt"
head -12 "$OUT/step_summary.txt"
