# round-6 GPU call 26: fused stem kernel phase isolation (no loads / no conv / no pooling builds)
set -o pipefail
export PYTHONPATH=$(pwd)
mkdir -p gpurun_out/r6
timeout -k 10 300 python scripts/stem_pool_iso.py --variants 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6/c26_variants.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "fused_stem" 2>&1 | tail -1
