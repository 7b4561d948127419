#!/bin/bash
# Real-training step rate: the CIFAR CLI (resnet_cifar_main.py, staged feeder,
# checkpoints/summaries on) at bs 128 and bs 32 -- single-GPU session, and the data-parallel
# engine on a single-rank process group (DRN_FORCE_DP=1) over the P2P all-reduce and over RCCL --
# next to bench.py's step for the same batch.
#   scripts/cli_step_rate.sh <outdir>
OUT=${1:-gpurun_out/cli_rate}
ROOT=$(pwd)
mkdir -p "$OUT"
export PYTHONPATH=$ROOT
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$OUT/data', 1000, learnable=True)" || exit 1
for bs in 128 32; do
  timeout -k 10 240 python -u bench.py --dataset cifar10 --batch_size $bs --steps 200 --warmup 20 \
    > "$OUT/bench_bs$bs.json" 2> "$OUT/bench_bs$bs.err" || { tail "$OUT/bench_bs$bs.err"; exit 1; }
  cat "$OUT/bench_bs$bs.json"
  for ar in single p2p rccl; do
    if [ $ar = single ]; then dp=0; arf=""; else dp=1; arf="--allreduce=$ar"; fi
    DRN_FORCE_DP=$dp timeout -k 10 240 python -u resnet_cifar_main.py --num_gpus=1 --train_data_path="$OUT/data" \
      --log_root="$OUT/ck_${ar}_$bs" --resnet_size=50 --batch_size=$bs --train_steps=1000 --log_every_n_steps=200 $arf \
      > "$OUT/cli_${ar}_bs$bs.log" 2>&1 || { tail -20 "$OUT/cli_${ar}_bs$bs.log"; exit 1; }
    echo "== bs $bs $ar"; grep -o 'step = [0-9]*.*steps/sec[^)]*' "$OUT/cli_${ar}_bs$bs.log" | tail -3
  done
done
