#!/bin/bash
#SBATCH --job-name=cifar_single
#SBATCH --time=6:00:00
#SBATCH --nodes=1
#SBATCH --gpus-per-node=1
#SBATCH --output=single_cifar.%j.log
# Serial (one GPU) CIFAR-10 ResNet-50 training (reference scripts/submit_cifar_daint_single.sh).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
DATA=${DATA_DIR:-${SCRATCH:-$HOME}/data}
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
${PYTHON:-python3} "$WORK_DIR/resnet_cifar_main.py" --train_data_path="$DATA" --log_root=./tmp/resnet_model \
  --train_dir=./tmp/resnet_model/train --dataset=cifar10 --num_gpus=1 --batch_size=${1:-128} --train_steps=80000
