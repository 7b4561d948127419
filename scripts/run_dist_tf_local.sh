#!/bin/bash
# One task of the local fake cluster (reference scripts/run_dist_tf_local.sh):
#   $1 job_name (ps|worker)  $2 task_index  $3 ps_hosts  $4 worker_hosts
# CPU, batch 10, synchronous all-reduce, 100 steps (the reference smoke configuration). Set
# TF_SCRIPT / TF_FLAGS to override; DATA_DIR for real CIFAR binaries (synthetic otherwise).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
TF_SCRIPT=${TF_SCRIPT:-$WORK_DIR/resnet_cifar_main.py}
DATA_FLAG="--synthetic_data=True"
[ -n "${DATA_DIR:-}" ] && DATA_FLAG="--train_data_path=${DATA_DIR}"
TF_FLAGS=${TF_FLAGS:-"$DATA_FLAG --log_root=./tmp/resnet_model --train_dir=./tmp/resnet_model/train
  --dataset=cifar10 --num_gpus=0 --batch_size=10 --sync_replicas=True --train_steps=100 --resnet_size=20"}
exec ${PYTHON:-python3} "$TF_SCRIPT" --job_name=$1 --task_index=$2 --ps_hosts=$3 --worker_hosts=$4 $TF_FLAGS
