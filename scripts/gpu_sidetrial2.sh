#!/bin/bash
# Side-stream trial on the P2P data-parallel graph step: tests, CIFAR DP benches, CLI (bs32, DP).
OUT=${1:-gpurun_out/st2}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_session_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > "$OUT/test.log" 2>&1
rc=$?; tail -3 "$OUT/test.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$OUT/test.log" | head -20; exit $rc; }
for bs in 32 128; do
  DRN_BENCH_DP=1 timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 50 --warmup 10 >> "$OUT/bench.jsonl" 2>> "$OUT/err.txt" || exit 1
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'): d=json.loads(l); c=d['config']; print(c['model'], c['global_batch'], d['ms_per_step'], c['hip_graph'], c['wgrad_side_stream'])"
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$ROOT/$OUT/data', 2000, learnable=True)" || exit 1
DRN_FORCE_DP=1 timeout -k 10 300 python resnet_cifar_main.py --num_gpus=1 --train_data_path="$ROOT/$OUT/data" --log_root="$ROOT/$OUT/ck" \
    --resnet_size=50 --batch_size=32 --train_steps=600 --log_every_n_steps=200 --allreduce=p2p > "$OUT/cli.log" 2>&1 || { tail -20 "$OUT/cli.log"; exit 1; }
grep -E "graph step|steps/sec" "$OUT/cli.log"
