# round-6 GPU call 36: publish-once BN finalize (one finalizing workgroup per large publishing
# launch, DRN_FIN_ONCE): GPU tests, bench A/B (3 rounds), remaining standalone finalize launches
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_executor_gpu.py -k moving_statistics > $O/c36_ms.txt 2>&1 || { tail -30 $O/c36_ms.txt; exit 1; }
tail -1 $O/c36_ms.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py > $O/c36_tests.txt 2>&1 || { tail -40 $O/c36_tests.txt; exit 1; }
tail -1 $O/c36_tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c36_x.json 2>> $O/c36.err || { tail $O/c36.err; exit 1; }
  echo "once $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c36_x.json | tr '\n' ' ')" | tee -a $O/c36_ab.txt
  DRN_FIN_ONCE=0 timeout -k 10 200 python bench.py > $O/c36_x.json 2>> $O/c36.err || { tail $O/c36.err; exit 1; }
  echo "launch $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c36_x.json | tr '\n' ' ')" | tee -a $O/c36_ab.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c36_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py --steps 10 --warmup 3 > $O/c36_prof.log 2>&1 || { tail -20 $O/c36_prof.log; exit 1; }
grep -i "fin_fwd\|finalize" $O/c36_prof/p_kernel_stats.csv | cut -c1-120
