set -o pipefail
export PYTHONPATH=$(pwd)
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_s6.log 2>&1 || { tail -20 gpurun_out/gputests_s6.log; exit 1; }
tail -2 gpurun_out/gputests_s6.log
timeout -k 10 240 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_s6.jsonl 2> gpurun_out/bench_s6.err && tail -1 gpurun_out/bench_s6.jsonl
