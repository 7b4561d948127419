# round-6 GPU call 27: fused stem (branch-free pooling, tap-0 repeat for out-of-image taps):
# correctness, isolated time, bench A/B vs DRN_STEM_POOL=0 (3 rounds)
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "fused_stem or maxpool" > $O/c27_tests.txt 2>&1 || { tail -40 $O/c27_tests.txt; exit 1; }
tail -1 $O/c27_tests.txt
timeout -k 10 120 python scripts/stem_pool_iso.py 2>&1 | grep -v amdgpu.ids | tee $O/c27_iso.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/c27_x.json 2>> $O/c27.err || { tail $O/c27.err; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"fused_stem_pool": [a-z]*' $O/c27_x.json | tr '\n' ' ')" | tee -a $O/c27_ab.txt
  DRN_STEM_POOL=0 timeout -k 10 200 python bench.py > $O/c27_x.json 2>> $O/c27.err || { tail $O/c27.err; exit 1; }
  echo "split $(grep -o '"ms_per_step": [0-9.]*\|"step_mode": "[a-z_]*"\|"fused_stem_pool": [a-z]*' $O/c27_x.json | tr '\n' ' ')" | tee -a $O/c27_ab.txt
done
