# round-6 GPU call 15: P2P data-parallel steps as native plans (runtime/plan.py) -- the P2P GPU
# tests, the single-rank P2P bench (mode times), the CIFAR CLI step rates; plus the isolated
# finalizing BN backward apply with the swizzled (tree) vs linear (r6db/oldbn) coefficient table.
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_session_gpu.py \
  tests/test_dp_gpu.py -k "p2p or session" > $O/c15_tests.txt 2>&1 || { tail -40 $O/c15_tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/c15_tests.txt | tail -20
for i in 1 2; do
  timeout -k 10 120 python scripts/bn_fin_iso.py --tag swizzled >> $O/c15_bn_iso.txt 2>&1 || exit 1
  DRN_KERNEL_LIB=$ROOT/r6db/oldbn/libdrn_kernels.so timeout -k 10 120 python scripts/bn_fin_iso.py --tag linear >> $O/c15_bn_iso.txt 2>&1 || exit 1
done
cat $O/c15_bn_iso.txt
for bs in 32 128; do
  DRN_BENCH_DP=1 timeout -k 10 240 python bench.py --dataset cifar10 --batch_size $bs --allreduce p2p --steps 200 --warmup 20 \
    > $O/c15_p2p_bench_bs$bs.json 2>> $O/c15.err || { tail $O/c15.err; exit 1; }
  cut -c1-400 $O/c15_p2p_bench_bs$bs.json
done
timeout -k 10 900 bash scripts/cli_step_rate.sh gpurun_out/r6/c15_cli > $O/c15_cli.txt 2>&1 || { tail -30 $O/c15_cli.txt; exit 1; }
cat $O/c15_cli.txt
