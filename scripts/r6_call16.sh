# round-6 GPU call 16: why the P2P data-parallel native plan runs 8-10 ms per CIFAR step (graph 2 ms):
# bench P2P plan modes with 4 and 8 hardware queues, then a kernel trace of the 4-queue plan run.
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
A="--dataset cifar10 --batch_size 32 --allreduce p2p --steps 50 --warmup 10 --graph 0 --plan 1"
DRN_BENCH_DP=1 timeout -k 10 200 python bench.py $A > $O/c16_q4.json 2>> $O/c16.err || { tail $O/c16.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"mode_trial_ms": {[^}]*}\|"hw_queues": "[0-9]*"' $O/c16_q4.json
DRN_BENCH_DP=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py $A > $O/c16_q8.json 2>> $O/c16.err || { tail $O/c16.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"mode_trial_ms": {[^}]*}\|"hw_queues": "[0-9]*"' $O/c16_q8.json
cd /tmp && export TMPDIR=/tmp
DRN_BENCH_DP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c16_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py $A > $O/c16_prof.log 2>&1 || { tail -20 $O/c16_prof.log; exit 1; }
echo prof done
