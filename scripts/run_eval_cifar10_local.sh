#!/bin/bash
# CIFAR-10 eval sidecar on a local machine (reference scripts/run_eval_cifar10_local.sh): polls
# ./tmp/resnet_model every --eval_interval_secs, writes Precision / Best Precision events.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
WORK_DIR="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$WORK_DIR${PYTHONPATH:+:$PYTHONPATH}"
DATA=${DATA_DIR:-$HOME/dataset}
${PYTHON:-python3} "$WORK_DIR/resnet_cifar_eval.py" --eval_data_path="$DATA/cifar-10-batches-bin/test_batch*" \
  --log_root=./tmp/resnet_model --eval_dir=./tmp/resnet_model/test --dataset=cifar10 --mode=eval --num_gpus=0 "$@"
