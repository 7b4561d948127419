#!/bin/bash
#SBATCH --job-name=cifar_eval
#SBATCH --time=0:30:00
#SBATCH --nodes=1
#SBATCH --gpus-per-node=1
#SBATCH --output=slurm_cifar_eval_%j.log
# One-shot CIFAR-10 evaluation of the latest checkpoint (reference
# scripts/submit_horovod_cifar_eval.sh with --eval_once=True).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
DATA=${DATA_DIR:-${SCRATCH:-$HOME}/data}
${PYTHON:-python3} "$WORK_DIR/resnet_cifar_eval.py" --eval_data_path="$DATA/cifar-10-batches-bin/test_batch*" \
  --log_root=./tmp/resnet_model --eval_dir=./tmp/resnet_model/test --dataset=cifar10 --mode=eval \
  --num_gpus=${NUM_GPUS:-1} --eval_once=True
