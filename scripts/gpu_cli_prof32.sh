#!/bin/bash
# Host profile of the CIFAR CLI at bs32 (graph step): where does the host spend a step?
OUT=${1:-gpurun_out/cp32}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$ROOT/$OUT/data', 2000, learnable=True)" || exit 1
timeout -k 10 300 python -m cProfile -o "$OUT/p.prof" resnet_cifar_main.py --num_gpus=1 --train_data_path="$ROOT/$OUT/data" \
  --log_root="$ROOT/$OUT/ck" --resnet_size=50 --batch_size=32 --train_steps=1000 --log_every_n_steps=250 > "$OUT/cli.log" 2>&1 || { tail "$OUT/cli.log"; exit 1; }
grep -E "graph step|steps/sec" "$OUT/cli.log"
python -c "import pstats; pstats.Stats('$OUT/p.prof').sort_stats('tottime').print_stats(25)" > "$OUT/prof.txt"
python -c "import pstats; pstats.Stats('$OUT/p.prof').sort_stats('cumulative').print_stats(40)" >> "$OUT/prof.txt"
grep -E "^\s+[0-9]" "$OUT/prof.txt" | head -60
