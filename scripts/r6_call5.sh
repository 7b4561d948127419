# round-6 GPU call 5: weight-gradient kernel tests (in-kernel split-K reduction), ImageNet copy-stream
# probe with the GPU_MAX_HW_QUEUES arms
set -o pipefail
mkdir -p gpurun_out/r6
export PYTHONPATH=$(pwd)
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "wgrad" > gpurun_out/r6/wgrad_tests.txt 2>&1 && \
timeout -k 10 700 python -u scripts/imagenet_copy_stream_probe.py > gpurun_out/r6/imagenet_copy_stream2.jsonl 2> gpurun_out/r6/imagenet_copy_stream2.err
