# round-6 GPU call 3: conv bound isolation incl. the no-loop variant and a tile-config sweep; plan + N>1 tests
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u scripts/conv_bound_iso.py --all --sweep --out gpurun_out/r6/conv_bound_iso_sweep.txt > gpurun_out/r6/conv_bound_iso_sweep.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py > gpurun_out/r6/plan_tests.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_dp_gpu.py -k "multirank or two_ranks_bitwise" > gpurun_out/r6/dp_tests.txt 2>&1
