# round-6 GPU call 33: final-tree verification -- full GPU test suite, smoke, benches (ResNet-50 x3,
# DP engine, WRN-50-2, CIFAR bs128 / bs32), early-SGD A/B (2 more rounds)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/c33_tests.txt 2>&1 || { tail -40 $O/c33_tests.txt; exit 1; }
tail -2 $O/c33_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/c33_smoke.txt 2>&1 || { tail $O/c33_smoke.txt; exit 1; }
tail -1 $O/c33_smoke.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py >> $O/c33_bench.jsonl 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
done
DRN_BENCH_DP=1 timeout -k 10 200 python bench.py >> $O/c33_dp.jsonl 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
timeout -k 10 300 python bench.py --resnet_size 50 --width 2 --batch_size 256 --steps 20 --warmup 5 >> $O/c33_wrn.jsonl 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
for bs in 128 32; do
  timeout -k 10 200 python bench.py --dataset cifar10 --batch_size $bs --steps 200 --warmup 20 >> $O/c33_cifar.jsonl 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
done
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/c33_x.json 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
  echo "early $(grep -o '"ms_per_step": [0-9.]*' $O/c33_x.json)" | tee -a $O/c33_ab.txt
  DRN_EARLY_SGD=0 timeout -k 10 200 python bench.py > $O/c33_x.json 2>> $O/c33.err || { tail $O/c33.err; exit 1; }
  echo "late $(grep -o '"ms_per_step": [0-9.]*' $O/c33_x.json)" | tee -a $O/c33_ab.txt
done
cut -c1-200 $O/c33_bench.jsonl $O/c33_dp.jsonl $O/c33_wrn.jsonl $O/c33_cifar.jsonl
