#!/bin/bash
#SBATCH --job-name=cifar_cpu
#SBATCH --time=4:00:00
#SBATCH --nodes=4
#SBATCH --output=cpu_cifar.%j.log
# CPU-cluster data-parallel CIFAR training over gloo (the reference's Cori KNL / MKL scripts,
# mkl-scripts/submit_ps_cifar_cori_dist.sh): one rank per node, global batch 128 split across
# the ranks as those scripts did. $1 TF_NUM_PS (unused) $2 ranks (default: nodes).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export WORK_DIR="$(cd "$HERE/.." && pwd)"
export TF_SCRIPT="${WORK_DIR}/resnet_cifar_main.py"
N=${2:-${SLURM_JOB_NUM_NODES:-1}}
export TF_NUM_PS=${1:-0} TF_NUM_WORKERS=$N TF_WORKER_PER_NODE=1
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-$(nproc)}
export TF_FLAGS="--train_data_path=${DATA_DIR:-${SCRATCH:-$HOME}/data} --log_root=./tmp/resnet_model
  --dataset=cifar10 --num_gpus=0 --batch_size=$(( 128 / N )) --sync_replicas=True --train_steps=80000"
mkdir -p ./logs/cpu-${N}-wk && cd ./logs/cpu-${N}-wk && "$HERE/run_dist_tf.sh"
