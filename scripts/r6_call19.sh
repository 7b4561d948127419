# round-6 GPU call 19: hardware-queue count 5 / 6 on the cases that 4 (ImageNet fed DP step) and 8
# (CIFAR P2P plan, CIFAR whole-step graph) each slow down
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
B="--dataset cifar10 --batch_size 32 --steps 100 --warmup 10"
for q in 5 6; do
  for cfg in "p2p_plan|1|--allreduce p2p --graph 0 --plan 1" "p2p_all|1|--allreduce p2p" "single|0|"; do
    IFS='|' read name dp args <<< "$cfg"
    DRN_BENCH_DP=$dp GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $B $args > $O/c19_x.json 2>> $O/c19.err || { tail $O/c19.err; exit 1; }
    echo "q$q $name $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"mode_trial_ms": {[^}]*}' $O/c19_x.json | tr '\n' ' ')" | tee -a $O/c19_modes.txt
  done
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python scripts/imagenet_copy_stream_probe.py --mode copystream > $O/c19_x.json 2>> $O/c19.err || { tail $O/c19.err; exit 1; }
  echo "q$q imagenet_copystream $(cat $O/c19_x.json)" | tee -a $O/c19_modes.txt
done
