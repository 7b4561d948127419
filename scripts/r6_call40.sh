# round-6 GPU call 40: fused stem weight gradient, fewer address / window instructions: op tests + isolated timing
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
export PYTHONPATH=$ROOT
timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_ops_gpu.py -k "stem_wgrad_pool" > $O/c40_op.txt 2>&1 || { tail -40 $O/c40_op.txt; exit 1; }
tail -1 $O/c40_op.txt
for v in 3 4; do DRN_STEM_WGRAD_POOL_NS=$v timeout -k 10 120 python -u scripts/stem_wgrad_pool_iso.py 2>&1 | grep -v amdgpu.ids >> $O/c40_iso.txt || { tail -20 $O/c40_iso.txt; exit 1; }; done
cat $O/c40_iso.txt
