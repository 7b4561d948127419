#!/bin/bash
# Multi-node (Slurm) or single-node launcher: training ranks + optional eval sidecar.
#
# Environment interface kept from the reference launchers (SURVEY §2.10;
# reference scripts/run_dist_tf_daint.sh:4-27, scripts/run_dist_train_eval_daint.sh:159-216):
#   TF_SCRIPT          training entry point (required)
#   TF_EVAL_SCRIPT     eval entry point (optional: runs as a sidecar process polling --log_root)
#   TF_FLAGS           flags for training;  TF_EVAL_FLAGS  flags for the eval sidecar
#   TF_NUM_PS          accepted for compatibility; parameter servers do not exist in the
#                      all-reduce engine (a notice is printed, no PS process is started)
#   TF_NUM_WORKERS     total training ranks (default: nodes x TF_WORKER_PER_NODE)
#   TF_WORKER_PER_NODE ranks (= GPUs) per node (default 8 on MI355X nodes, 1 without GPUs)
#   TF_PS_PER_NODE, TF_PS_IN_WORKER   accepted, ignored
#   PYTHON             interpreter (default python3)
# Logs: ./worker.$JOB.<host>-<rank>.log per rank, ./eval.$JOB.log; child PIDs in ./.drn_pids
# (scripts/kill.sh stops exactly those). Every rank resumes from the latest checkpoint in
# --log_root, so resubmitting the same job continues training.
set -u
PYTHON=${PYTHON:-python3}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(cd "$HERE/.." && pwd)"
export PYTHONPATH="$REPO${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0

if [ -z "${TF_SCRIPT:-}" ]; then
  echo "Set the variable TF_SCRIPT"
  exit 1
fi
JOB=${SLURM_JOB_ID:-local$$}
if [ -n "${TF_NUM_PS:-}" ] && [ "${TF_NUM_PS}" != "0" ]; then
  echo "[drn] TF_NUM_PS=${TF_NUM_PS}: parameter servers are not used by the all-reduce engine; starting workers only"
fi

# node list
if [ -n "${SLURM_JOB_NODELIST:-}" ]; then
  NODES=($(scontrol show hostnames "$SLURM_JOB_NODELIST"))
else
  NODES=("$(hostname)")
fi
NNODES=${#NODES[@]}
if [ -z "${TF_WORKER_PER_NODE:-}" ]; then
  NGPU=$($PYTHON -c "import torch; print(torch.cuda.device_count())" 2>/dev/null || echo 0)
  TF_WORKER_PER_NODE=$(( NGPU > 0 ? NGPU : 1 ))
fi
TF_NUM_WORKERS=${TF_NUM_WORKERS:-$(( NNODES * TF_WORKER_PER_NODE ))}
WNODES=$(( (TF_NUM_WORKERS + TF_WORKER_PER_NODE - 1) / TF_WORKER_PER_NODE ))
if [ "$WNODES" -gt "$NNODES" ]; then
  echo "The number of allocated nodes is not enough for TF_NUM_WORKERS=$TF_NUM_WORKERS"
  exit 1
fi
PER_NODE=$(( TF_NUM_WORKERS < TF_WORKER_PER_NODE ? TF_NUM_WORKERS : TF_WORKER_PER_NODE ))
if [ "$WNODES" -gt 1 ] && [ $(( TF_NUM_WORKERS % TF_WORKER_PER_NODE )) -ne 0 ]; then
  echo "TF_NUM_WORKERS must be a multiple of TF_WORKER_PER_NODE across nodes"
  exit 1
fi
MASTER_ADDR=${MASTER_ADDR:-${NODES[0]}}
[ "$NNODES" -eq 1 ] && MASTER_ADDR=127.0.0.1
MASTER_PORT=${MASTER_PORT:-$(( 29500 + (${SLURM_JOB_ID:-$$} % 1000) ))}
: > .drn_pids

LAUNCH="$PYTHON -m distributed_resnet_tensorflow_amd.parallel.launch --nproc $PER_NODE --nnodes $WNODES \
  --master_addr $MASTER_ADDR --master_port $MASTER_PORT --log_dir . --tag $JOB --pid_file .drn_pids"
echo "[drn] $TF_NUM_WORKERS workers on $WNODES node(s) x $PER_NODE, rendezvous $MASTER_ADDR:$MASTER_PORT"

TRAIN_PIDS=()
if [ "$WNODES" -gt 1 ]; then
  for (( n=0; n<WNODES; n++ )); do
    srun --nodelist="${NODES[$n]}" -N 1 -n 1 --exclusive $LAUNCH --node_rank $n "$TF_SCRIPT" ${TF_FLAGS:-} &
    TRAIN_PIDS+=($!)
  done
else
  $LAUNCH --node_rank 0 "$TF_SCRIPT" ${TF_FLAGS:-} &
  TRAIN_PIDS+=($!)
fi
printf '%s\n' "${TRAIN_PIDS[@]}" >> .drn_pids

# eval sidecar: on the node after the workers when one is free, else locally (CPU or a GPU the
# workers do not use)
if [ -n "${TF_EVAL_SCRIPT:-}" ]; then
  if [ "$NNODES" -gt "$WNODES" ] && [ -n "${SLURM_JOB_NODELIST:-}" ]; then
    srun --nodelist="${NODES[$WNODES]}" -N 1 -n 1 $PYTHON "$TF_EVAL_SCRIPT" ${TF_EVAL_FLAGS:-} > eval.$JOB.log 2>&1 &
  else
    $PYTHON "$TF_EVAL_SCRIPT" ${TF_EVAL_FLAGS:-} > eval.$JOB.log 2>&1 &
  fi
  EVAL_PID=$!
  echo $EVAL_PID >> .drn_pids
fi

# wait for the training ranks; then stop the sidecar (it polls forever unless --eval_once)
rc=0
for pid in "${TRAIN_PIDS[@]}"; do
  wait "$pid" || rc=$?
done
if [ -n "${EVAL_PID:-}" ]; then
  sleep "${DRN_EVAL_GRACE:-5}"
  kill "$EVAL_PID" 2>/dev/null
  wait "$EVAL_PID" 2>/dev/null
fi
exit $rc
