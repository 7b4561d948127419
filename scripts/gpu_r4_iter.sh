#!/bin/bash
# Round-4 iteration check: targeted GPU tests, ResNet-50 + CIFAR benches, CIFAR bs32 profile.
#   TESTS="<pytest selection>" scripts/gpu_r4_iter.sh <outdir>
OUT=${1:-gpurun_out/it}
export PYTHONPATH=$(pwd)
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_ops_gpu.py} -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 python bench.py >> "$OUT/rn50.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  for bs in 128 32; do
    timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/cifar.jsonl" 2>> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
  done
done
python3 -c "
import json,sys
for f in ('rn50','cifar'):
    for l in open('$OUT/'+f+'.jsonl'):
        d=json.loads(l); print(f, d['config']['per_gpu_batch'], d['ms_per_step'], d['value'], d['config']['hip_graph'])"
[ -n "$NOPROF" ] && exit 0
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o step --output-format csv -- \
  python3 "$ROOT/bench.py" --dataset cifar10 --batch_size 32 --steps 5 --warmup 2 --graph 0 > "$ROOT/$OUT/prof.log" 2>&1 || { tail "$ROOT/$OUT/prof.log"; exit 1; }
cd "$ROOT"
python3 scripts/prof_step.py "$OUT/prof/step_kernel_trace.csv" 1000 > "$OUT/cifar32_step_summary.txt"
head -8 "$OUT/cifar32_step_summary.txt"
