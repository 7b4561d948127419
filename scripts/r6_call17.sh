# round-6 GPU call 17: kernel trace of the slow P2P data-parallel plan (8 hardware queues)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
A="--dataset cifar10 --batch_size 32 --allreduce p2p --steps 30 --warmup 5 --graph 0 --plan 1"
cd /tmp && export TMPDIR=/tmp
DRN_BENCH_DP=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c17_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py $A > $O/c17_prof.log 2>&1 || { tail -20 $O/c17_prof.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"mode_trial_ms": {[^}]*}' $O/c17_prof.log
