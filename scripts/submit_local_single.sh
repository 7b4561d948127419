#!/bin/bash
# Serial CPU smoke run (reference scripts/submit_mac_single.sh): batch 10, CPU.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
DATA_FLAG="--synthetic_data=True"
[ -n "${DATA_DIR:-}" ] && DATA_FLAG="--train_data_path=${DATA_DIR}"
${PYTHON:-python3} "$WORK_DIR/resnet_cifar_main.py" $DATA_FLAG --log_root=./tmp/resnet_model \
  --train_dir=./tmp/resnet_model/train --dataset=cifar10 --num_gpus=0 --batch_size=10 \
  --train_steps=${TRAIN_STEPS:-80000} --resnet_size=${RESNET_SIZE:-20}
