#!/bin/bash
# Real-training (CIFAR CLI) step rate without a profiler, P2P graph path and RCCL eager path,
# plus a cProfile of the P2P run's host loop.
OUT=${1:-gpurun_out/cli}
ROOT=$(pwd)
mkdir -p "$OUT"
export PYTHONPATH=$ROOT DRN_FORCE_DP=1
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$ROOT/$OUT/data', 2000, learnable=True)" || exit 1
for ar in p2p rccl; do
  timeout -k 10 300 python "$ROOT/resnet_cifar_main.py" --num_gpus=1 --train_data_path="$ROOT/$OUT/data" --log_root="$ROOT/$OUT/ck_$ar" \
    --resnet_size=50 --batch_size=128 --train_steps=400 --log_every_n_steps=100 --allreduce=$ar > "$OUT/$ar.log" 2>&1 || { tail -20 "$OUT/$ar.log"; exit 1; }
  grep "steps/sec" "$OUT/$ar.log"
done
timeout -k 10 300 python -m cProfile -o "$OUT/p2p.prof" "$ROOT/resnet_cifar_main.py" --num_gpus=1 --train_data_path="$ROOT/$OUT/data" --log_root="$ROOT/$OUT/ck_prof" \
    --resnet_size=50 --batch_size=128 --train_steps=400 --log_every_n_steps=100 --allreduce=p2p > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python -c "import pstats; pstats.Stats('$OUT/p2p.prof').sort_stats('tottime').print_stats(35)" > "$OUT/p2p_prof.txt"
python -c "import pstats; pstats.Stats('$OUT/p2p.prof').sort_stats('cumulative').print_stats(45)" >> "$OUT/p2p_prof.txt"
head -60 "$OUT/p2p_prof.txt"
