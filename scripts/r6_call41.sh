# round-6 GPU call 41: final-tree verification after the stream-K publish guard -- full GPU test
# suite, smoke, benches (ResNet-50 x3, DP engine, CIFAR bs128 / bs32), plan-mode step trace
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/c41_tests.txt 2>&1 || { tail -40 $O/c41_tests.txt; exit 1; }
tail -2 $O/c41_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/c41_smoke.txt 2>&1 || { tail $O/c41_smoke.txt; exit 1; }
tail -1 $O/c41_smoke.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py >> $O/c41_bench.jsonl 2>> $O/c41.err || { tail $O/c41.err; exit 1; }
done
DRN_BENCH_DP=1 timeout -k 10 200 python bench.py >> $O/c41_dp.jsonl 2>> $O/c41.err || { tail $O/c41.err; exit 1; }
for bs in 128 32; do
  timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 200 --warmup 20 >> $O/c41_cifar.jsonl 2>> $O/c41.err || { tail $O/c41.err; exit 1; }
done
cut -c1-200 $O/c41_bench.jsonl $O/c41_dp.jsonl $O/c41_cifar.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c41_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py --steps 10 --warmup 3 > $O/c41_prof.log 2>&1 || { tail -20 $O/c41_prof.log; exit 1; }
cd $ROOT
python3 scripts/prof_step.py $O/c41_prof/p_kernel_trace.csv > $O/c41_step_summary.txt || true
python3 scripts/step_streams.py $O/c41_prof/p_kernel_trace.csv > $O/c41_streams.txt || true
head -8 $O/c41_streams.txt
