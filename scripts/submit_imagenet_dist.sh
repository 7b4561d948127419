#!/bin/bash
#SBATCH --job-name=imagenet
#SBATCH --time=24:00:00
#SBATCH --nodes=1
#SBATCH --gpus-per-node=8
#SBATCH --output=dist_imagenet.%j.log
# ImageNet ResNet-50 v2 data-parallel training + eval sidecar (reference
# scripts/submit_imagenet_daint_dist.sh). $1 TF_NUM_PS (unused) $2 ranks $3 per-rank batch
# $4 wipe. Set SYNTHETIC=1 for synthetic data of the benchmark shape.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export WORK_DIR="$(cd "$HERE/.." && pwd)"
export TF_SCRIPT="${WORK_DIR}/resnet_imagenet_main.py"
export TF_EVAL_SCRIPT="${WORK_DIR}/resnet_imagenet_eval.py"
DATA=${DATA_DIR:-${SCRATCH:-$HOME}/data/imagenet}
export BATCH_SIZE=${3:-128}
SYN=""
[ "${SYNTHETIC:-0}" = "1" ] && SYN="--synthetic_data=True"
export TF_FLAGS="--train_data_path=${DATA} --log_root=./tmp/resnet_model --train_dir=./tmp/resnet_model/train
  --dataset=imagenet --num_gpus=1 --batch_size=${BATCH_SIZE} --sync_replicas=True --train_steps=${TRAIN_STEPS:-120000} ${SYN}"
export TF_EVAL_FLAGS="--eval_data_path=${DATA} --log_root=./tmp/resnet_model --eval_dir=./tmp/resnet_model/test
  --dataset=imagenet --mode=eval --num_gpus=0"
[ "${SYNTHETIC:-0}" = "1" ] && unset TF_EVAL_SCRIPT
export TF_NUM_PS=${1:-0}
export TF_NUM_WORKERS=${2:-8}
DIR=./logs/${TF_NUM_PS}-ps-${TF_NUM_WORKERS}-wk-batch-${BATCH_SIZE}-imagenet-log
if [ -n "$4" ]; then rm -rf "$DIR"; else rm -f "$DIR"/*.log; fi
mkdir -p "$DIR" && cd "$DIR" && "$HERE/run_dist_train_eval.sh"
