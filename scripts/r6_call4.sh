# round-6 GPU call 4: ImageNet copy-stream probe, CIFAR CLI step rates with the
# dedicated graph stream (item 5), WRN-50-2 re-baseline with DP diagnostics (item 7)
set -o pipefail
mkdir -p gpurun_out/r6
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u scripts/imagenet_copy_stream_probe.py > gpurun_out/r6/imagenet_copy_stream.jsonl 2> gpurun_out/r6/imagenet_copy_stream.err && \
timeout -k 10 900 bash scripts/cli_step_rate.sh gpurun_out/r6/cli_rate > gpurun_out/r6/cli_rate.txt 2>&1 && \
timeout -k 10 300 python bench.py --width 2 --batch_size 256 > gpurun_out/r6/wrn.jsonl 2> gpurun_out/r6/wrn.err && \
DRN_BENCH_DP=1 timeout -k 10 300 python bench.py --width 2 --batch_size 256 >> gpurun_out/r6/wrn.jsonl 2>> gpurun_out/r6/wrn.err && \
DRN_BENCH_DP=1 timeout -k 10 300 python bench.py >> gpurun_out/r6/rn50_dp.jsonl 2>> gpurun_out/r6/wrn.err
