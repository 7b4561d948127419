# round-6 GPU call 43: optimizer after the side stream's max-pool backward (DRN_SGD_AFTER_POOL) A/B
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
DRN_SGD_AFTER_POOL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_plan_gpu.py tests/test_executor_gpu.py > $O/c43_tests.txt 2>&1 || { tail -30 $O/c43_tests.txt; exit 1; }
tail -1 $O/c43_tests.txt
for i in 1 2 3; do
  DRN_SGD_AFTER_POOL=1 timeout -k 10 200 python bench.py > $O/c43_x.json 2>> $O/c43.err || { tail $O/c43.err; exit 1; }
  echo "after_pool $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c43_x.json | tr '\n' ' ')" | tee -a $O/c43_ab.txt
  timeout -k 10 200 python bench.py > $O/c43_x.json 2>> $O/c43.err || { tail $O/c43.err; exit 1; }
  echo "default    $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c43_x.json | tr '\n' ' ')" | tee -a $O/c43_ab.txt
done
