#!/bin/bash
# Root-causing the held-out precision spread of tests/test_cli_gpu.py (learnable fake CIFAR):
# train resnet-8 like the test (3 seeds), then evaluate the checkpoint with the moving BN
# statistics on (a) the held-out test file and (b) the training files. A gap on (b) points at the
# moving statistics / eval path; no gap on (b) but one on (a) is generalisation.
#   scripts/probes/cifar_eval_probe.sh <outdir>
OUT=${1:-gpurun_out/cifar_probe}
mkdir -p "$OUT"
export PYTHONPATH=$(pwd)
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$OUT/data', 1000, learnable=True)" || exit 1
for seed in 1 2 3; do
  ck=$OUT/ck$seed
  timeout -k 10 300 python -u resnet_cifar_main.py --num_gpus=1 --train_data_path=$OUT/data --log_root=$ck \
    --resnet_size=8 --batch_size=128 --train_steps=2000 --log_every_n_steps=500 --seed=$seed > $OUT/train$seed.log 2>&1 || { tail $OUT/train$seed.log; exit 1; }
  grep "precision =" $OUT/train$seed.log | tail -2
  for what in test train; do
    if [ $what = test ]; then pat="$OUT/data/cifar-10-batches-bin/test_batch*"; else pat="$OUT/data/cifar-10-batches-bin/data_batch_1*"; fi
    timeout -k 10 200 python -u resnet_cifar_eval.py --mode=eval --eval_once=True --num_gpus=1 \
      --eval_data_path="$pat" --log_root=$ck --eval_dir=$OUT/ev_${what}_$seed --resnet_size=8 \
      --eval_batch_count=10 > $OUT/eval_${what}_$seed.log 2>&1 || { tail $OUT/eval_${what}_$seed.log; exit 1; }
    echo "seed $seed $what: $(grep -o 'precision: [0-9.]*' $OUT/eval_${what}_$seed.log | tail -1)"
  done
done
