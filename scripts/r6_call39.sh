# round-6 GPU call 39: packed-stem weight gradient with the max-pool backward fused into its dY
# operand (DRN_STEM_WGRAD_POOL): op tests, isolated timing, executor tests, bench A/B
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_ops_gpu.py -k "stem_wgrad_pool or packed_stem" > $O/c39_op.txt 2>&1 || { tail -40 $O/c39_op.txt; exit 1; }
tail -1 $O/c39_op.txt
for v in 3 4 5; do DRN_STEM_WGRAD_POOL_NS=$v timeout -k 10 120 python -u scripts/stem_wgrad_pool_iso.py >> $O/c39_iso.txt 2>&1 || { tail -20 $O/c39_iso.txt; exit 1; }; done
cat $O/c39_iso.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py > $O/c39_tests.txt 2>&1 || { tail -40 $O/c39_tests.txt; exit 1; }
tail -1 $O/c39_tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c39_x.json 2>> $O/c39.err || { tail $O/c39.err; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c39_x.json | tr '\n' ' ')" | tee -a $O/c39_ab.txt
  DRN_STEM_WGRAD_POOL=0 timeout -k 10 200 python bench.py > $O/c39_x.json 2>> $O/c39.err || { tail $O/c39.err; exit 1; }
  echo "two   $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c39_x.json | tr '\n' ' ')" | tee -a $O/c39_ab.txt
done
