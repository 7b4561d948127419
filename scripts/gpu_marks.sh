#!/bin/bash
# Side-stream marks every 1 / 2 / 4 weight gradients: tests (every 3), then ResNet-50 + CIFAR benches.
OUT=${1:-gpurun_out/marks}
export PYTHONPATH=$(pwd)
DB=$(pwd)/distributed_resnet_tensorflow_amd/ops/tune_db.json
mkdir -p "$OUT"
DRN_MARK_EVERY=3 timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/tests.log" | head -20; exit $rc; }
bash scripts/gpu_env_ab.sh "$OUT" ${ROUNDS:-4} "m1=DRN_TUNE_DB=$DB DRN_MARK_EVERY=1" "m2=DRN_TUNE_DB=$DB DRN_MARK_EVERY=2" \
  "m4=DRN_TUNE_DB=$DB DRN_MARK_EVERY=4" || exit 1
for m in 1 4; do
  for bs in 128 32; do
    line=$(DRN_MARK_EVERY=$m timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 2>> "$OUT/err.txt") || exit 1
    echo "cifar m$m bs$bs $(echo "$line" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a "$OUT/ab.txt"
  done
done
