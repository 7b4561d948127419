# round-6 GPU call 9: the reverted (round-5) kernels + round-6 runtime: bench x2, step profile,
# CIFAR CLI step rates, plan / N>1 rehearsal tests
set -o pipefail
mkdir -p gpurun_out/r6
export PYTHONPATH=$(pwd)
timeout -k 10 300 python bench.py > gpurun_out/r6/c9_bench.jsonl 2> gpurun_out/r6/c9_bench.err && \
timeout -k 10 300 python bench.py >> gpurun_out/r6/c9_bench.jsonl 2>> gpurun_out/r6/c9_bench.err && \
bash scripts/gpu_prof_step.sh gpurun_out/r6/prof > gpurun_out/r6/c9_prof.txt 2>&1 && \
timeout -k 10 900 bash scripts/cli_step_rate.sh gpurun_out/r6/cli_rate2 > gpurun_out/r6/cli_rate2.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py > gpurun_out/r6/c9_plan_tests.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_dp_gpu.py > gpurun_out/r6/c9_dp_tests.txt 2>&1
