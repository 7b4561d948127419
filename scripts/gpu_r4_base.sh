#!/bin/bash
# Round-4 baseline on one GPU box: smoke, default bench, single-rank DP bench (RCCL eager / CIFAR P2P graph),
# CIFAR benches, then a kernel-trace profile of the ResNet-50 step. Stops at the first failure.
OUT=${1:-gpurun_out/r4base}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
set -o pipefail
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py >> "$OUT/bench_rn50.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py >> "$OUT/bench_rn50_dp.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
done
for bs in 128 32; do
  timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench_cifar.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench_cifar_dp.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
done
cat "$OUT"/bench_*.jsonl
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --graph 0 > "$ROOT/$OUT/prof.log" 2>&1 || { tail "$ROOT/$OUT/prof.log"; exit 1; }
cd "$ROOT"
python3 scripts/prof_step.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/step_summary.txt"
python3 scripts/step_streams.py "$OUT/prof/step_kernel_trace.csv" > "$OUT/streams.txt" || true
head -40 "$OUT/step_summary.txt"; cat "$OUT/streams.txt"
