#!/bin/bash
# GPU end-to-end smoke of the reference-named entry points on one MI355X (fake CIFAR data).
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/e2e}
mkdir -p $OUT
python -c "import sys; sys.path.insert(0,'.'); from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$OUT/data', 512)"
timeout -k 10 300 python resnet_cifar_main.py --num_gpus=1 --train_data_path=$OUT/data --log_root=$OUT/ck \
  --eval_dir=$OUT/ev --batch_size=128 --train_steps=200 --log_every_n_steps=50 > $OUT/train.log 2>&1
timeout -k 10 300 python resnet_cifar_eval.py --mode=eval --num_gpus=1 --eval_once=True --eval_data_path=$OUT/data \
  --log_root=$OUT/ck --eval_dir=$OUT/ev --eval_batch_count=5 > $OUT/eval.log 2>&1
tail -4 $OUT/train.log; tail -1 $OUT/eval.log
