#!/bin/bash
# CIFAR CLI step rate with the feeder prefetch on a worker thread vs inline (bs32 / bs128).
OUT=${1:-gpurun_out/apf}
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p "$OUT"
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$ROOT/$OUT/data', 2000, learnable=True)" || exit 1
for r in 1 2; do rm -rf "$OUT"/ck_* ;
  for a in 1 0; do
    for bs in 32 128; do
      DRN_ASYNC_PREFETCH=$a timeout -k 10 300 python resnet_cifar_main.py --num_gpus=1 --train_data_path="$ROOT/$OUT/data" \
        --log_root="$ROOT/$OUT/ck_${r}_${a}_$bs" --resnet_size=50 --batch_size=$bs --train_steps=800 --log_every_n_steps=400 \
        > "$OUT/cli_${r}_${a}_$bs.txt" 2>&1 || { tail -20 "$OUT/cli_${r}_${a}_$bs.txt"; exit 1; }
      echo "$r async=$a bs=$bs $(grep "step = 800" "$OUT/cli_${r}_${a}_$bs.txt" | grep -o '([0-9.]* steps/sec')" | tee -a "$OUT/ab.txt"
    done
  done
done
rm -rf "$OUT"/ck_* "$OUT"/data; grep -h "graph step" "$OUT"/cli_*.txt | cut -c 25-
