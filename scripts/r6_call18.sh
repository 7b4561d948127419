# round-6 GPU call 18: P2P without the report stream (comm waits on both compute streams):
# P2P GPU tests, then CIFAR bs32 step modes at 4 and 8 hardware queues (P2P plan only / P2P all
# modes / single GPU)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_session_gpu.py \
  tests/test_dp_gpu.py -k "p2p" > $O/c18_tests.txt 2>&1 || { tail -40 $O/c18_tests.txt; exit 1; }
grep -E "passed|failed" $O/c18_tests.txt | tail -2
B="--dataset cifar10 --batch_size 32 --steps 100 --warmup 10"
for q in 4 8; do
  for cfg in "p2p_plan|1|--allreduce p2p --graph 0 --plan 1" "p2p_all|1|--allreduce p2p" "single|0|"; do
    IFS='|' read name dp args <<< "$cfg"
    DRN_BENCH_DP=$dp GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $B $args > $O/c18_x.json 2>> $O/c18.err || { tail $O/c18.err; exit 1; }
    echo "q$q $name $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"mode_trial_ms": {[^}]*}' $O/c18_x.json | tr '\n' ' ')" | tee -a $O/c18_modes.txt
  done
done
