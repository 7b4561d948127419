#!/bin/bash
# ImageNet eval (reference scripts/run_local.sh).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
${PYTHON:-python3} "$WORK_DIR/resnet_imagenet_eval.py" --eval_data_path="${DATA_DIR:-$HOME/data/imagenet}" \
  --log_root=./tmp/resnet_model --eval_dir=./tmp/resnet_model/test --dataset=imagenet --mode=eval \
  --num_gpus=${NUM_GPUS:-1} "$@"
