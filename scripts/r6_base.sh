set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python bench.py > gpurun_out/r6/base_bench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py > gpurun_out/r6/plan_tests.txt 2>&1 && \
timeout -k 10 300 python scripts/conv3x3_bench.py --all > gpurun_out/r6/base_conv3x3.txt 2>&1
