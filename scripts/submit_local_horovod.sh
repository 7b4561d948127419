#!/bin/bash
# All-reduce ("Horovod") training on one machine (reference scripts/submit-horovod-train-mac.sh,
# which ran `mpirun -np 4`): N ranks through the drn launcher; GPUs when present, else CPU/gloo.
#   $1: ranks (default 4)   $2: per-rank batch (default 32)
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
NG=$(${PYTHON:-python3} -c "import torch; print(1 if torch.cuda.device_count() else 0)" 2>/dev/null || echo 0)
DATA_FLAG="--synthetic_data=True"
[ -n "${DATA_DIR:-}" ] && DATA_FLAG="--train_data_path=${DATA_DIR}"
: > .drn_pids
${PYTHON:-python3} -m distributed_resnet_tensorflow_amd.parallel.launch --nproc ${1:-4} --pid_file .drn_pids \
  "$WORK_DIR/resnet_cifar_main_horovod.py" --use_horovod=True $DATA_FLAG --log_root=./tmp/resnet_model \
  --train_dir=./tmp/resnet_model/train --dataset=cifar10 --num_gpus=$NG --batch_size=${2:-32} \
  --sync_replicas=True --train_steps=${TRAIN_STEPS:-80000}
