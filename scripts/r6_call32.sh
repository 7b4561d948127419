# round-6 GPU call 32: early optimizer for every block but the first (DRN_EARLY_SGD): executor /
# plan / bench-geometry / session tests, bench A/B (3 rounds)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py tests/test_session_gpu.py > $O/c32_tests.txt 2>&1 || { tail -40 $O/c32_tests.txt; exit 1; }
tail -1 $O/c32_tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c32_x.json 2>> $O/c32.err || { tail $O/c32.err; exit 1; }
  echo "early $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c32_x.json | tr '\n' ' ')" | tee -a $O/c32_ab.txt
  DRN_EARLY_SGD=0 timeout -k 10 200 python bench.py > $O/c32_x.json 2>> $O/c32.err || { tail $O/c32.err; exit 1; }
  echo "late $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c32_x.json | tr '\n' ' ')" | tee -a $O/c32_ab.txt
done
