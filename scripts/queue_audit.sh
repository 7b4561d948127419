#!/bin/bash
# HW-queue audit of REAL training on one GPU: the CIFAR CLI with its real
# staged feeder, run through the data-parallel engine on a single-rank process group
# (DRN_FORCE_DP=1) -- RCCL (eager step, high-priority main stream, RCCL's stream, the weight-
# gradient side stream, the feeder's copy stream) and the P2P all-reduce (whole-step graph, its
# comm stream). Kernel traces -> scripts/step_streams.py: the side stream must still overlap the
# main stream (no serialised regime: 4 HW queues per process).
#   scripts/queue_audit.sh <outdir>
OUT=${1:-gpurun_out/queue_audit}
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
export PYTHONPATH=$ROOT DRN_FORCE_DP=1
python -c "from distributed_resnet_tensorflow_amd.data.cifar import write_fake_cifar; write_fake_cifar('$ROOT/$OUT/data', 1000, learnable=True)" || exit 1
cd /tmp && export TMPDIR=/tmp
for ar in rccl p2p; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/$ar" -o tr --output-format csv -- \
    python3 "$ROOT/resnet_cifar_main.py" --num_gpus=1 --train_data_path="$ROOT/$OUT/data" --log_root="$ROOT/$OUT/ck_$ar" \
    --resnet_size=50 --batch_size=128 --train_steps=40 --log_every_n_steps=20 --allreduce=$ar \
    > "$ROOT/$OUT/$ar.log" 2>&1 || { tail -20 "$ROOT/$OUT/$ar.log"; exit 1; }
  echo "== $ar"
  python3 "$ROOT/scripts/step_streams.py" "$ROOT/$OUT/$ar/tr_kernel_trace.csv" | tee "$ROOT/$OUT/$ar.streams.txt"
done
