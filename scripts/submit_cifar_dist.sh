#!/bin/bash
#SBATCH --job-name=cifar
#SBATCH --time=2:30:00
#SBATCH --nodes=1
#SBATCH --gpus-per-node=8
#SBATCH --output=dist_cifar.%j.log
# CIFAR-10 ResNet-50 data-parallel training + eval sidecar on MI355X nodes
# (reference scripts/submit_cifar_daint_dist.sh). Arguments as in the reference:
#   $1: TF_NUM_PS (accepted, unused)  $2: TF_NUM_WORKERS (ranks = GPUs)  $3: per-rank batch (128)
#   $4: any value -> wipe the previous run's directory (else resume from its checkpoints)
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export WORK_DIR="$(cd "$HERE/.." && pwd)"
export TF_SCRIPT="${WORK_DIR}/resnet_cifar_main.py"
export TF_EVAL_SCRIPT="${WORK_DIR}/resnet_cifar_eval.py"
export DATASET=${DATASET:-cifar10}
DATA=${DATA_DIR:-${SCRATCH:-$HOME}/data}
export BATCH_SIZE=${3:-128}
export TF_FLAGS="--train_data_path=${DATA} --log_root=./tmp/resnet_model --train_dir=./tmp/resnet_model/train
  --dataset=${DATASET} --num_gpus=1 --batch_size=${BATCH_SIZE} --sync_replicas=True --train_steps=80000"
export TF_EVAL_FLAGS="--eval_data_path=${DATA}/cifar-10-batches-bin/test_batch* --log_root=./tmp/resnet_model
  --eval_dir=./tmp/resnet_model/test --dataset=${DATASET} --mode=eval --num_gpus=0"
export TF_NUM_PS=${1:-0}
export TF_NUM_WORKERS=${2:-8}
DIR=./logs/${TF_NUM_PS}-ps-${TF_NUM_WORKERS}-wk-batch-${BATCH_SIZE}-${DATASET}-log
if [ -n "$4" ]; then
  echo "remove previous checkpoints"
  rm -rf "$DIR"
else
  rm -f "$DIR"/*.log
fi
mkdir -p "$DIR" && cd "$DIR" && "$HERE/run_dist_train_eval.sh"
