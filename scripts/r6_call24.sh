# round-6 GPU call 24: persistent fused stem conv + max-pool: correctness, isolated time, bench A/B
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "fused_stem" > $O/c24_tests.txt 2>&1 || { tail -40 $O/c24_tests.txt; exit 1; }
tail -1 $O/c24_tests.txt
timeout -k 10 120 python scripts/stem_pool_iso.py 2>&1 | grep -v amdgpu.ids | tee $O/c24_iso.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/c24_x.json 2>> $O/c24.err || { tail $O/c24.err; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"fused_stem_pool": [a-z]*' $O/c24_x.json | tr '\n' ' ')" | tee -a $O/c24_ab.txt
  DRN_STEM_POOL=0 timeout -k 10 200 python bench.py > $O/c24_x.json 2>> $O/c24.err || { tail $O/c24.err; exit 1; }
  echo "split $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"fused_stem_pool": [a-z]*' $O/c24_x.json | tr '\n' ' ')" | tee -a $O/c24_ab.txt
done
