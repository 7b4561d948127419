# round-6 GPU call 20: final P2P buckets on the current stream: P2P tests, CIFAR bs32 P2P / single
# step modes (4 hardware queues, the box default), kernel trace of the P2P plan
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dp_gpu.py -k "p2p" > $O/c20_tests.txt 2>&1 || { tail -40 $O/c20_tests.txt; exit 1; }
grep -E "passed|failed" $O/c20_tests.txt | tail -2
B="--dataset cifar10 --batch_size 32 --steps 100 --warmup 10"
for cfg in "p2p_all|1|--allreduce p2p" "single|0|" "p2p_all|1|--allreduce p2p" "single|0|"; do
  IFS='|' read name dp args <<< "$cfg"
  DRN_BENCH_DP=$dp timeout -k 10 200 python bench.py $B $args > $O/c20_x.json 2>> $O/c20.err || { tail $O/c20.err; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"mode_trial_ms": {[^}]*}\|"hw_queues": "[0-9]*"' $O/c20_x.json | tr '\n' ' ')" | tee -a $O/c20_modes.txt
done
cd /tmp && export TMPDIR=/tmp
DRN_BENCH_DP=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c20_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py --dataset cifar10 --batch_size 32 --allreduce p2p --steps 30 --warmup 5 --graph 0 --plan 1 > $O/c20_prof.log 2>&1 || { tail -20 $O/c20_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c20_prof1 -o p --output-format csv -- \
  python3 $ROOT/bench.py --dataset cifar10 --batch_size 32 --steps 30 --warmup 5 --graph 0 --plan 1 > $O/c20_prof1.log 2>&1 || { tail -20 $O/c20_prof1.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"mode_trial_ms": {[^}]*}' $O/c20_prof.log $O/c20_prof1.log
cd $ROOT
# the fed ImageNet data-parallel step at the box's 4 hardware queues: copy stream at normal vs high priority
for m in "copystream|0" "copystream|-1" "synthetic|0" "copystream|-1"; do
  IFS='|' read mode pr <<< "$m"
  DRN_COPY_STREAM_PRIORITY=$pr timeout -k 10 400 python scripts/imagenet_copy_stream_probe.py --mode $mode > $O/c20_x.json 2>> $O/c20.err || { tail $O/c20.err; exit 1; }
  echo "prio$pr $(grep '^{' $O/c20_x.json)" | tee -a $O/c20_imagenet.txt
done
