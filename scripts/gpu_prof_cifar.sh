#!/bin/bash
# Kernel-trace profile of the CIFAR ResNet-50 bs32 / bs128 graph steps.
OUT=${1:-gpurun_out/pcifar}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for bs in 32 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof$bs" -o step --output-format csv -- \
    python3 "$ROOT/bench.py" --dataset cifar10 --batch_size $bs --steps 10 --warmup 5 > "$ROOT/$OUT/prof$bs.log" 2>&1 || { tail "$ROOT/$OUT/prof$bs.log"; exit 1; }
  python3 "$ROOT/scripts/step_streams.py" "$ROOT/$OUT/prof$bs/step_kernel_trace.csv" > "$ROOT/$OUT/streams$bs.txt" || true
  python3 "$ROOT/scripts/prof_step.py" "$ROOT/$OUT/prof$bs/step_kernel_trace.csv" > "$ROOT/$OUT/summary$bs.txt" || true
  head -12 "$ROOT/$OUT/streams$bs.txt"
done
