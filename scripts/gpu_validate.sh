#!/bin/bash
# Full validation on one GPU box (run from the repo root): every GPU test, smoke, the benches
# (ResNet-50, single-rank data-parallel engine, CIFAR bs128 / bs32, Wide-ResNet-50-2) and a
# kernel-trace profile of one ResNet-50 step. Stops at the first failure.
#   scripts/gpu_validate.sh <outdir> [skip-tests]
OUT=${1:-gpurun_out/val}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
set -o pipefail
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1
  rc=$?; tail -3 "$OUT/tests.txt"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.txt" | head -20; exit $rc; }
fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py >> "$OUT/bench_rn50.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py >> "$OUT/bench_rn50_dp.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
done
for bs in 128 32; do
  timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench_cifar.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench_cifar_dp.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
done
timeout -k 10 300 python bench.py --width 2 --batch_size 256 --steps 10 --warmup 3 >> "$OUT/bench_wrn.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cut -c1-240 "$OUT"/bench_*.jsonl
bash scripts/gpu_prof_step.sh "$OUT"
