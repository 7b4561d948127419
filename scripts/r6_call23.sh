# round-6 GPU call 23: fused stem conv + max-pool (csrc/kernels/stem_pool.hip): correctness, the
# executor / plan tests on the ImageNet topology, bench A/B against DRN_STEM_POOL=0, kernel times
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ops_gpu.py \
  -k "fused_stem or packed_stem or maxpool" > $O/c23_tests.txt 2>&1 || { tail -40 $O/c23_tests.txt; exit 1; }
grep -E "passed|failed" $O/c23_tests.txt | tail -1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_executor_gpu.py \
  tests/test_plan_gpu.py tests/test_bench_geometry_gpu.py > $O/c23_tests2.txt 2>&1 || { tail -40 $O/c23_tests2.txt; exit 1; }
tail -1 $O/c23_tests2.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c23_x.json 2>> $O/c23.err || { tail $O/c23.err; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"fused_stem_pool": [a-z]*' $O/c23_x.json | tr '\n' ' ')" | tee -a $O/c23_ab.txt
  DRN_STEM_POOL=0 timeout -k 10 200 python bench.py > $O/c23_x.json 2>> $O/c23.err || { tail $O/c23.err; exit 1; }
  echo "split $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"' $O/c23_x.json | tr '\n' ' ')" | tee -a $O/c23_ab.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c23_prof -o p --output-format csv -- \
  python3 $ROOT/bench.py --steps 10 --warmup 3 > $O/c23_prof.log 2>&1 || { tail -20 $O/c23_prof.log; exit 1; }
grep -i "stem\|maxpool" $O/c23_prof/p_kernel_stats.csv | cut -c1-150
