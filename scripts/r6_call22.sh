# round-6 GPU call 22: final P2P data-parallel path (inline reductions for small gradients, native
# plans, no report stream) and the high-priority ImageNet copy stream: P2P / session / feeder GPU
# tests, P2P bench, CIFAR CLI step rates
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_dp_gpu.py tests/test_session_gpu.py \
  > $O/c22_tests.txt 2>&1 || { tail -40 $O/c22_tests.txt; exit 1; }
grep -E "passed|failed" $O/c22_tests.txt | tail -2
for bs in 32 128; do
  DRN_BENCH_DP=1 timeout -k 10 240 python bench.py --dataset cifar10 --batch_size $bs --allreduce p2p --steps 200 --warmup 20 \
    > $O/c22_p2p_bench_bs$bs.json 2>> $O/c22.err || { tail $O/c22.err; exit 1; }
  echo "p2p bs$bs $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"mode_trial_ms": {[^}]*}' $O/c22_p2p_bench_bs$bs.json | tr '\n' ' ')"
done
timeout -k 10 900 bash scripts/cli_step_rate.sh gpurun_out/r6/c22_cli > $O/c22_cli.txt 2>&1 || { tail -30 $O/c22_cli.txt; exit 1; }
cat $O/c22_cli.txt
grep -h "step:" gpurun_out/r6/c22_cli/cli_*.log
