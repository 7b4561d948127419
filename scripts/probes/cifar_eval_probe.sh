#!/bin/bash
# Root-causing the held-out precision spread of tests/test_cli_gpu.py (learnable fake CIFAR):
# train resnet-8 like the test (3 seeds; constant LR 0.1 for 2000 steps, and the reference
# schedule compressed 20x: 0.1 -> 0.01 at 2000 -> 0.001 at 3000, 3500 steps), then evaluate the
# checkpoint with the moving BN statistics on (a) the held-out test file and (b) the training
# files, and run scripts/probes/bn_eval_diag.py (moving vs batch vs recalibrated statistics).
#   scripts/probes/cifar_eval_probe.sh <outdir>
OUT=${1:-gpurun_out/cifar_probe}
mkdir -p "$OUT"
export PYTHONPATH=$(pwd)
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$OUT/data', 1000, learnable=True)" || exit 1
B=$OUT/data/cifar-10-batches-bin
for cfg in const sched; do
  if [ $cfg = const ]; then extra="--train_steps=2000"; else extra="--train_steps=3500 --lr_schedule_scale=0.05"; fi
  for seed in 1 2 3; do
    ck=$OUT/ck_${cfg}_$seed
    timeout -k 10 300 python -u resnet_cifar_main.py --num_gpus=1 --train_data_path=$OUT/data --log_root=$ck \
      --resnet_size=8 --batch_size=128 $extra --log_every_n_steps=500 --seed=$seed > $OUT/train_${cfg}_$seed.log 2>&1 \
      || { tail $OUT/train_${cfg}_$seed.log; exit 1; }
    for what in test train; do
      if [ $what = test ]; then pat="$B/test_batch*"; else pat="$B/data_batch_1*"; fi
      timeout -k 10 200 python -u resnet_cifar_eval.py --mode=eval --eval_once=True --num_gpus=1 \
        --eval_data_path="$pat" --log_root=$ck --eval_dir=$OUT/ev_${cfg}_${what}_$seed --resnet_size=8 \
        --eval_batch_count=10 > $OUT/eval_${cfg}_${what}_$seed.log 2>&1 || { tail $OUT/eval_${cfg}_${what}_$seed.log; exit 1; }
      echo "$cfg seed $seed $what: $(grep -o 'precision: [0-9.]*' $OUT/eval_${cfg}_${what}_$seed.log | tail -1)"
    done
    timeout -k 10 200 python -u scripts/probes/bn_eval_diag.py $ck "$B/data_batch_*" 8 || exit 1
  done
done
