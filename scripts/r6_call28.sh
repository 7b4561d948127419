# round-6 GPU call 28: the stem's max-pool backward on the side stream (deferred tail): executor /
# plan / bench-geometry tests, bench A/B vs DRN_POOL_BWD_SIDE=0 (3 rounds)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py > $O/c28_tests.txt 2>&1 || { tail -40 $O/c28_tests.txt; exit 1; }
tail -1 $O/c28_tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c28_x.json 2>> $O/c28.err || { tail $O/c28.err; exit 1; }
  echo "side $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c28_x.json | tr '\n' ' ')" | tee -a $O/c28_ab.txt
  DRN_POOL_BWD_SIDE=0 timeout -k 10 200 python bench.py > $O/c28_x.json 2>> $O/c28.err || { tail $O/c28.err; exit 1; }
  echo "main $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c28_x.json | tr '\n' ' ')" | tee -a $O/c28_ab.txt
done
