# round-6 GPU call 37: stream-K publish-once guard (fin-once experiment removed): GPU tests + bench
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_ops_gpu.py -k "publishes_once or streamk" > $O/c37_sk.txt 2>&1 || { tail -30 $O/c37_sk.txt; exit 1; }
tail -1 $O/c37_sk.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py > $O/c37_tests.txt 2>&1 || { tail -40 $O/c37_tests.txt; exit 1; }
tail -1 $O/c37_tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c37_x.json 2>> $O/c37.err || { tail $O/c37.err; exit 1; }
  cat $O/c37_x.json >> $O/c37_bench.jsonl
  grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c37_x.json | tr '\n' ' '; echo
done
