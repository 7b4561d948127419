#!/bin/bash
# scripts/cli_host_probe.py over the CIFAR CLI, bs 32: single-GPU session and the data-parallel
# engine over RCCL on a single-rank group (each session's own step-mode trial picks the mode).
OUT=${1:-gpurun_out/cli_hp}
ROOT=$(pwd)
mkdir -p "$OUT"
export PYTHONPATH=$ROOT
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$OUT/data', 1000, learnable=True)" || exit 1
for cfg in "single 0" "rccl 1"; do
  set -- $cfg
  arf=""; [ $1 = rccl ] && arf="--allreduce=rccl"
  DRN_FORCE_DP=$2 timeout -k 10 240 python -u scripts/cli_host_probe.py --num_gpus=1 --train_data_path="$OUT/data" \
    --log_root="$OUT/ck_$1" --resnet_size=50 --batch_size=32 --train_steps=600 --log_every_n_steps=200 $arf \
    > "$OUT/$1.log" 2>&1 || { tail -20 "$OUT/$1.log"; exit 1; }
  echo "#### $1"; grep -o 'step: .*\|step = 600.*steps/sec[^)]*' "$OUT/$1.log"; sed -n '/== host probe/,$p' "$OUT/$1.log"
done
