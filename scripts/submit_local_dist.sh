#!/bin/bash
# Local fake cluster (reference scripts/submit_mac_dist.sh; README.md:86 calls it
# submit_local_dist.sh): one process per "host", distinct localhost ports standing in for
# distinct hosts, using the reference's --job_name/--task_index/--ps_hosts/--worker_hosts CLI.
# PS processes print a notice and exit; the workers train with the all-reduce engine.
#   $1: number of PS (default 1)  $2: number of workers (default 2)
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
TF_NUM_PS=${1:-1}
TF_NUM_WORKER=${2:-2}
PS_HOSTS=$(for i in $(seq 0 $((TF_NUM_PS - 1))); do printf 'localhost:%s,' $((2230 + i)); done)
PS_HOSTS=${PS_HOSTS%,}
WK_HOSTS=$(for i in $(seq 0 $((TF_NUM_WORKER - 1))); do printf 'localhost:%s,' $((2220 + i)); done)
WK_HOSTS=${WK_HOSTS%,}
: > .drn_pids
echo "starting PSs..."
for i in $(seq 0 $((TF_NUM_PS - 1))); do
  "$HERE/run_dist_tf_local.sh" ps $i "$PS_HOSTS" "$WK_HOSTS" > ps$i.log 2>&1 &
  echo $! >> .drn_pids
done
echo "starting WORKERs..."
for i in $(seq 0 $((TF_NUM_WORKER - 1))); do
  "$HERE/run_dist_tf_local.sh" worker $i "$PS_HOSTS" "$WK_HOSTS" > wk$i.log 2>&1 &
  echo $! >> .drn_pids
done
wait
